"""Guard for the compiler miscompile class these kernels have met (DESIGN.md
§5.3): LLVM losing a value that is live across a divergent branch on the lanes
of the other arm.  Round 3 traced one instance to the pre-RA MachineSink; in
round 5 the round-4 WPaxos same-key P2b absorb (PXS_WP_ABSORB=1) miscompiles
with the round-4 flags (MachineSink off): at step 2 of the wp_crash case the Flaky ppm
(200000) of replica 3's P1b send lands in the slot of every instance the P1a
created.  Whether the wrong code appears depends on the exact source, so
build() compiles the whole library from a pinned commit (__graft_entry__.GUARD_COMMIT;
only its C ABI, include/paxisim.h, must equal the tree's) into
paxi_amd/guard/libpaxisim_absorb.so, a live reproducer; this test asserts that it diverges from the oracle and that
the product library does not, on the same case (tools/sink_guard.py), and that
neither does the variant built without LLVM's SDWA peephole nor the variant
whose send_begin is the product's one-exit form (the source-level fix)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402


def test_guard_variants_are_declared():
    assert ge.GUARDS["absorb"] == ["-DPXS_WP_ABSORB=1", "-mllvm", "-disable-machine-sink"]
    assert ge.GUARDS["absorb_nosdwa"][-1] == "-amdgpu-sdwa-peephole=false"
    assert ge.GUARDS["absorb_oneexit"] == ge.GUARDS["absorb"] and ge.GUARD_SEND_PATCH == {"absorb_oneexit"}
    assert ge.GUARD_UNIT in ge.HIP_SOURCES


def _run(lib, *cases):
    env = dict(os.environ, PAXISIM_LIB=os.path.join(ROOT, lib))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sink_guard.py"), *cases], env=env, cwd=ROOT,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_absorb_variant_diverges_and_product_does_not():
    var_lib = ge.guard_lib("absorb")
    assert os.path.exists(os.path.join(ROOT, var_lib)), "guard variant not built: run __graft_entry__.build()"
    prod = _run(ge.HIP_LIB)
    var = _run(var_lib, "wp_crash")
    print("product", prod, "\nvariant", var)
    assert not any(prod["diverged"].values()), prod
    assert var["diverged"]["wp_crash"], var                   # the live reproducer
    assert var["build_id"] == prod["build_id"] + f"+guard:absorb@{ge.GUARD_COMMIT}"


@pytest.mark.gpu
def test_absorb_without_sdwa_peephole_matches_oracle():
    """The pass bisection's finding: the same absorb source,
    built without LLVM's SDWA peephole, does not diverge."""
    lib = ge.guard_lib("absorb_nosdwa")
    assert os.path.exists(os.path.join(ROOT, lib)), "guard variant not built: run __graft_entry__.build()"
    res = _run(lib, "wp_crash")
    assert not res["diverged"]["wp_crash"], res


@pytest.mark.gpu
def test_absorb_with_one_exit_send_matches_oracle():
    """The source-level fix the product ships (sim_core.h PXS_SEND_ONE_EXIT):
    the pinned reproducer with the tree's one-exit send_begin in place of its
    early-return one does not diverge, with the same flags as the reproducer."""
    lib = ge.guard_lib("absorb_oneexit")
    assert os.path.exists(os.path.join(ROOT, lib)), "guard variant not built: run __graft_entry__.build()"
    res = _run(lib, "wp_crash")
    assert not res["diverged"]["wp_crash"], res
