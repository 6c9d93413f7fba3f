"""The round-5 miscompile, named at the instruction level, on
the ISA build() leaves in build/guard/isa (the pinned reproducer's unit and
its variants, compiled with line tables, which leave the code unchanged).

tools/repro/isa_slot_check.py finds the VGPR that carries x.slot into
wp_unbind's instance store and lists every write to it inside the P1b's
send_begin.  In the reproducer the Flaky branch's fault-table scan (scripted,
paxisim_dev.h) loads into that register, while the copy of x.slot is made
before the branch and again only on the send path: a lane whose P1b is
dropped stores the scan's value as its slot - the wrong instances the GPU
test sees.  The SDWA-free and one-exit builds, and the product's unit, keep
the slot register out of the scan.  Skipped where build() has not run."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ISA = os.path.join(ROOT, ge.GUARD_OBJ, "isa")
PINNED = os.path.join(ROOT, ge.GUARD_OBJ, "src", ge.GUARD_COMMIT, "paxi_amd", "csrc")


def check(name, csrc):
    path = os.path.join(ISA, name + ".s")
    if not os.path.exists(path):
        pytest.skip(f"{path} not built (run __graft_entry__.build())")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "repro", "isa_slot_check.py"), path, csrc],
                         capture_output=True, text=True, check=True)
    return json.loads(out.stdout)


def test_reproducer_clobbers_the_slot_register_in_the_flaky_scan():
    r = check("absorb", PINNED)
    assert r["slot_registers"] and r["slot_clobbered_by_fault_scan"], r
    assert all(w["at"].startswith("paxisim_dev.h") for w in r["writes"]), r


@pytest.mark.parametrize("name", ["absorb_nosdwa", "absorb_oneexit", "product"])
def test_fixed_builds_keep_the_slot_register_out_of_the_scan(name):
    csrc = {"absorb_nosdwa": PINNED,
            "absorb_oneexit": os.path.join(ROOT, ge.GUARD_OBJ, "src", ge.GUARD_COMMIT + "_oneexit", "paxi_amd", "csrc"),
            "product": os.path.join(ROOT, ge.CSRC)}[name]
    r = check(name, csrc)
    assert r["slot_registers"] and r["p1b_send_begin_instructions"] > 0, r
    assert not r["slot_clobbered_by_fault_scan"], r
