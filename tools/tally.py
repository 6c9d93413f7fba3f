"""Diagnostic: HBM requests per delivered message by access class (DESIGN.md
§5.10), from a PXS_TALLY build of the library (paxisim_dev.h tally_at).

Every instrumented load or store adds, per wave instruction, its active lanes
and the distinct 128-B lines (loads) or 32-B sectors (stores) they touch - the
requests it sends to L2.  This runs a BASELINE config's workload (bench.workload)
at a reduced cluster count through the bench's warm-up, enables the counters,
runs one bench step, and prints per class: lane accesses and requests per
delivered message, and the bytes those requests would move if none hit in L2
(128 B per line read, 32 B per sector written, DESIGN.md §5.6's calibration).
Compare the total with the measured FETCH_SIZE / WRITE_SIZE per message.

  PAXISIM_LIB=var/v_tally.so python tools/tally.py <config> [clusters] [out.json]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from paxi_amd.sim import Simulation, load_library  # noqa: E402

# TallyClass (paxisim_dev.h), in order
CLASSES = ["record load", "record store", "instance load", "instance store", "entry load", "entry store",
           "replica row load", "replica row store", "counter atomic", "kv load", "kv store", "forwards table",
           "pending list", "checkpoint / digest", "agreement ring", "reply value", "ghost table", "link state",
           "other (request side table, policy)"]
TALLY_PER = 48


def main():
    cfg_id = int(sys.argv[1])
    clusters = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    a = argparse.Namespace(window=None, mbox=None, kv=1, history=512, clusters=clusters, sim_steps=None,
                           warmup=5, steps=1, crash_step=None, fz=1)
    for k, v in bench.DEFAULTS[cfg_id].items():
        if getattr(a, k, None) is None:
            setattr(a, k, v)
    a.crash_step = a.warmup * a.sim_steps
    os.environ.setdefault("PAXISIM_LAUNCH_STEPS", str(bench.launch_steps(cfg_id)))
    cfg, wl, fp, faults, _ = bench.workload(cfg_id, clusters, 0, 0, a)
    L = load_library()
    L.paxisim_dbg_enable.argtypes = [C.c_void_p]
    L.paxisim_dbg_read.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    g = Simulation(cfg, wl, fp, faults)
    for _ in range(a.warmup):
        g.step(a.sim_steps)
    g.sync()
    assert L.paxisim_dbg_enable(g.h) == 0
    s0 = g.stats().as_dict()
    g.step(a.sim_steps)
    g.sync()
    s1 = g.stats().as_dict()
    nb = (g.cfg.clusters + 63) // 64
    # the library sizes the buffer by its slot capacity C (>= clusters)
    cap = max(nb, 1) * 2
    buf = (C.c_ulonglong * (cap * 16 * TALLY_PER))()
    assert L.paxisim_dbg_read(g.h, buf) == 0
    msgs = s1["delivered_total"] - s0["delivered_total"]
    rows = {}
    tot_rd = tot_wr = 0.0
    for ci, name in enumerate(CLASSES):
        row = {}
        for kind, off, unit in (("load", 0, 128), ("store", 2, 32)):
            lanes = sum(buf[b * 16 * TALLY_PER + 4 * ci + off] for b in range(cap))
            units = sum(buf[b * 16 * TALLY_PER + 4 * ci + off + 1] for b in range(cap))
            if not lanes:
                continue
            byts = units * unit / max(1, msgs)
            row[kind] = {"lane_accesses_per_msg": lanes / max(1, msgs), "requests_per_msg": units / max(1, msgs),
                         "unit": f"{unit}-B {'line' if unit == 128 else 'sector'}",
                         "bytes_per_msg_if_no_l2_hits": byts}
            if kind == "store":
                tot_wr += byts
            else:
                tot_rd += byts
        if row:
            rows[name] = row
    g.close()
    out = {"config": cfg_id, "clusters": clusters, "window": [a.warmup * a.sim_steps, (a.warmup + 1) * a.sim_steps],
           "messages": msgs, "classes": rows, "read_bytes_per_msg_if_no_l2_hits": tot_rd,
           "write_bytes_per_msg_if_no_l2_hits": tot_wr,
           "note": "every ghost-table reference (load or store) counts as a line read"}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")


if __name__ == "__main__":
    main()
