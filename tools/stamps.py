"""Diagnostic: per-phase cycle breakdown of the step kernel (PXS_STAMPS build).
usage: python tools/stamps.py <clusters> <warmup_steps> <steps> [config (2..5), default 2]"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from paxi_amd import abi
import bench

L = C.CDLL(os.path.join(ROOT, "paxi_amd", os.environ.get("PAXISIM_STAMPS_LIB", "libpaxisim_stamps.so")))
abi.declare(L, "paxisim")
L.paxisim_step.argtypes = [C.c_void_p, C.c_uint32]
L.paxisim_dbg_enable.argtypes = [C.c_void_p]
L.paxisim_dbg_read.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
clusters, warm, steps = (int(a) for a in sys.argv[1:4])
config = int(sys.argv[4]) if len(sys.argv) > 4 else 2
args = argparse.Namespace(window=bench.DEFAULTS[config]["window"], mbox=bench.DEFAULTS[config]["mbox"], history=512, kv=1,
                          crash_step=1000)
cfg, wl, fp, faults, _ = bench.workload(config, clusters, 0, 0, args)
cfg.steps_per_launch = 50
h = C.c_void_p()
assert L.paxisim_create(C.byref(cfg), C.byref(wl), C.byref(fp) if fp is not None else None, C.byref(h)) == 0, \
    L.paxisim_last_error()
for f in faults:
    assert L.paxisim_fault_add(h, C.byref(f)) == 0
assert L.paxisim_dbg_enable(h) == 0
if warm:
    L.paxisim_step(h, warm)
nb = (clusters + 63) // 64
DBG_PER = 48
buf = (C.c_ulonglong * (nb * 16 * DBG_PER))()
L.paxisim_dbg_read(h, buf)
L.paxisim_step(h, steps)
L.paxisim_dbg_read(h, buf)
N = sum(cfg.npz[i] for i in range(cfg.n_zones))
print(f"config {config}: {clusters} clusters, steps [{warm}, {warm + steps})")
for r in range(N):
    tot = [0] * 12
    for b in range(nb):
        # dbg is indexed by replica
        for k in range(12):
            tot[k] += buf[(b * 16 + r) * DBG_PER + k]
    st = max(1, tot[5])
    print(f"replica {r}: per wave-step setup {tot[0]/st:8.0f} loop {tot[1]/st:8.0f} barrier {tot[2]/st:8.0f} cyc;"
          f" lane-0 trips {tot[3]/st:5.2f}, records/lane {tot[4]/st/64:5.2f};"
          f" per lane-0 trip: pick+prefetch {tot[6]/max(1,tot[3]):6.0f} dispatch {tot[7]/max(1,tot[3]):6.0f}"
          f" head {tot[8]/max(1,tot[3]):6.0f} flush {tot[9]/max(1,tot[3]):6.0f}"
          f" rest {(tot[1]-tot[6]-tot[7]-tot[8]-tot[9]-tot[10]-tot[11])/max(1,tot[3]):6.0f};"
          f" per step: stage {tot[10]/st:7.0f} after lane 0 done (other lanes trips) {tot[11]/st:7.0f}")
NAMES = {0: "client req+bind", 1: "REQUEST", 2: "REPLY", 3: "P1A", 4: "P1B", 6: "P2A", 7: "P2B", 8: "P3",
         9: "GET", 10: "GETREPLY", 11: "SET", 12: "SETREPLY", 13: "LEADERCHG", 14: "bind", 15: "unbind"}
if config in (2, 4):   # Multi-Paxos: sub-handler regions in the slots ABD / WPaxos use (paxisim_dev.h PXS_SUB_T*)
    NAMES.update({5: " P3>exec", 9: " P2B>exec", 10: " P2B>entry", 11: " P2B>ack", 12: "absorb loop", 13: "send flush"})
print("handler paths (cycles per wave-step, runs per wave-step, cycles per run), summed over replicas:")
cyc = [0] * 16
runs = [0] * 16
steps = 0
for r in range(N):
    for b in range(nb):
        q = (b * 16 + r) * DBG_PER
        steps += buf[q + 5]
        for k in range(16):
            cyc[k] += buf[q + 16 + k]
            runs[k] += buf[q + 32 + k]
steps = max(1, steps)
for k in range(16):
    if runs[k]:
        print(f"  {NAMES.get(k, k):>16}: {cyc[k]/steps:9.0f} cyc/wave-step  {runs[k]/steps:6.2f} runs/wave-step"
              f"  {cyc[k]/runs[k]:8.0f} cyc/run")
