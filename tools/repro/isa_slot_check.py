"""The round-5 miscompile at the instruction level, checked on
the pinned reproducer's ISA.

Usage: python tools/repro/isa_slot_check.py <unit.s> <pinned csrc dir>
(the unit compiled with --offload-device-only -S -gline-tables-only; the
line tables do not change the code: the reproducer's 49,189 instructions are
identical with and without them).

In the 9-replica serial WPaxos kernel, wp_unbind (wpaxos_kernel.h) stores a
kpaxos instance as `global_store_dwordx4 v[..], v[B:B+3]` = {ballot, slot,
execute, meta}, so v(B+1) carries x.slot into the store.  paxos_handle_p1a
(paxos_kernel.h) sends its P1b through send_begin (sim_core.h), whose Flaky
test scans the scripted fault table (scripted(), paxisim_dev.h) inside a
divergent branch.  This lists, inside that send_begin, every instruction that
writes the slot register, with its source line and whether it lies in the
fault-table scan.  The reproducer's signature: the slot register is written by
the scan's loads (the Flaky branch's lanes), while its copy of x.slot is made
before the branch and again only on the send path, so a lane whose P1b the
Flaky draw drops reaches the store with the scan's last value.  Prints JSON."""
import json
import os
import re
import sys

LOC = re.compile(r"\s*\.loc\s+\d+\s+\d+\s+\d+.*;\s*(\S.*)$")


def parse(path):
    out, chain = [], ""
    for n, line in enumerate(open(path), 1):
        m = LOC.match(line)
        if m:
            chain = m.group(1).strip()
            continue
        s = line.split(";")[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        out.append((n, s, chain))
    return out


def src_line(csrc, fname, needle):
    for k, line in enumerate(open(os.path.join(csrc, fname)), 1):
        if needle in line:
            return k
    raise SystemExit(f"{needle!r} not in {fname}")


def writes(instr, reg):
    """Does the instruction write VGPR number `reg` (first operand)?"""
    op, _, rest = instr.partition(" ")
    if not op.startswith("v_") or op.startswith(("v_cmp", "v_readlane", "v_readfirstlane", "v_writelane")):
        if not op.startswith(("global_load", "buffer_load", "flat_load", "ds_read")):
            return False
    dst = rest.split(",")[0].strip()
    m = re.fullmatch(r"v(\d+)", dst)
    if m:
        return int(m.group(1)) == reg
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", dst)
    return bool(m) and int(m.group(1)) <= reg <= int(m.group(2))


def main():
    path, csrc = sys.argv[1], sys.argv[2]
    ins = parse(path)
    unbind = src_line(csrc, "wpaxos_kernel.h", "] = make_uint4(x.ballot, (uint32_t)x.slot")
    p1b_send = src_line(csrc, "paxos_kernel.h", "send_begin<NT>(P, x, bal_id(mb)")
    stores = [(n, s) for n, s, ch in ins
              if s.startswith("global_store_dwordx4") and re.match(rf"(\S*/)?wpaxos_kernel\.h:{unbind}:", ch)]
    slot_regs = sorted({int(re.search(r"v\[(\d+):\d+\]\s*,\s*off", s).group(1)) + 1 for _, s in stores}
                       if stores else set())
    tag = re.compile(rf"(^|/)paxos_kernel\.h:{p1b_send}:")
    region = [(n, s, ch) for n, s, ch in ins if tag.search(ch)]
    res = {"unit": path, "unbind_stores": [n for n, _ in stores], "slot_registers": [f"v{r}" for r in slot_regs],
           "p1b_send_begin_instructions": len(region), "writes": []}
    for r in slot_regs:
        for n, s, ch in region:
            if writes(s, r):
                inner = ch.split(" @[")[0].split("paxi_amd/csrc/")[-1]
                res["writes"].append({"line": n, "instr": s, "at": inner,
                                      "in_fault_scan": inner.startswith("paxisim_dev.h")})
    res["slot_clobbered_by_fault_scan"] = any(w["in_fault_scan"] for w in res["writes"])
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
