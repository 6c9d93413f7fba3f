"""CPU-side checks of the C-ABI boundary: the HIP library loads and exports
every symbol include/paxisim.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "paxisim.h")).read()
    return sorted(set(re.findall(r"\b(paxisim_[a-z_]+)\s*\(", hdr)))


def test_header_declares_api():
    syms = declared_symbols()
    for s in ["paxisim_create", "paxisim_step", "paxisim_stats_get", "paxisim_read_state",
              "paxisim_check", "paxisim_destroy", "paxisim_last_error", "paxisim_fault_add"]:
        assert s in syms


def test_library_exports_all_declared():
    from paxi_amd import sim
    lib = os.path.join(ROOT, "paxi_amd", "libpaxisim.so")
    assert os.path.exists(lib), "build() first"
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (paxisim_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    assert set(sim.EXPORTED) <= exported


def test_library_loads_and_reports_version():
    from paxi_amd import abi, sim
    L = sim.load_library()
    assert L.paxisim_abi_version() == abi.ABI_VERSION


def test_struct_layout_matches_header():
    """Compile a tiny C probe against paxisim.h and compare sizeof/offsetof with ctypes."""
    from paxi_amd import abi
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "paxisim.h"
int main(void){
 printf("%zu %zu %zu %zu %zu %zu\n", sizeof(paxisim_config), sizeof(paxisim_workload),
   sizeof(paxisim_fault_process), sizeof(paxisim_fault), sizeof(paxisim_replica_state), sizeof(paxisim_stats));
 printf("%zu %zu %zu\n", offsetof(paxisim_config, clusters), offsetof(paxisim_replica_state, delivered),
   offsetof(paxisim_stats, flagged));
 return 0;}
'''
    import tempfile
    d = tempfile.mkdtemp()
    open(os.path.join(d, "p.c"), "w").write(src)
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", os.path.join(d, "p"), os.path.join(d, "p.c")],
                   check=True)
    out = subprocess.run([os.path.join(d, "p")], capture_output=True, text=True, check=True).stdout.split()
    got = [int(x) for x in out]
    want = [ctypes.sizeof(abi.Config), ctypes.sizeof(abi.Workload), ctypes.sizeof(abi.FaultProcess),
            ctypes.sizeof(abi.Fault), ctypes.sizeof(abi.ReplicaState), ctypes.sizeof(abi.Stats),
            abi.Config.clusters.offset, abi.ReplicaState.delivered.offset, abi.Stats.flagged.offset]
    assert got == want


def test_create_without_gpu_fails_loudly():
    """No device here: the product path must refuse, never fall back to the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from paxi_amd import abi, sim
    with pytest.raises(sim.PaxisimError):
        sim.Simulation(abi.make_config(clusters=4), abi.make_workload())


def test_quorum_predicates_match_the_oracle():
    """paxisim_quorum (the kernels' own predicate, built for the host) equals the
    oracle's restatement of quorum.go:55-119 for every kind, mask and layout."""
    import oracle_lib as ol
    from paxi_amd import abi, sim
    for npz in ([3], [5], [2, 2], [3, 3, 3], [2, 3, 4], [4, 4, 4, 4]):
        for fz in (0, 1, 2):
            cfg = abi.make_config(npz=npz, fz=fz)
            n = sum(npz)
            masks = range(1 << n) if n <= 9 else range(0, 1 << n, 37)
            for kind in range(8):
                for m in masks:
                    assert sim.quorum(cfg, kind, m) == ol.quorum(kind, npz, m, fz), (npz, fz, kind, m)
