"""Diagnostic: per-phase cycle breakdown of the step kernel (PXS_STAMPS build).
usage: python tools/stamps.py <clusters> <warmup_steps> <steps>"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from paxi_amd import abi

L = C.CDLL(os.path.join(ROOT, "paxi_amd", "libpaxisim_stamps.so"))
abi.declare(L, "paxisim")
L.paxisim_step.argtypes = [C.c_void_p, C.c_uint32]
L.paxisim_dbg_enable.argtypes = [C.c_void_p]
L.paxisim_dbg_read.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
clusters, warm, steps = (int(a) for a in sys.argv[1:4])
cfg = abi.make_config(npz=[5], clusters=clusters, seed=42, window=16, mbox_cap=32, max_delay=4, steps_per_launch=50)
wl = abi.make_workload(outstanding=8, target=0)
fp = abi.make_fault_process(drop_ppm=1000, drop_len=50, slow_ppm=1000, slow_len=50, slow_min=1, slow_max=4)
h = C.c_void_p()
assert L.paxisim_create(C.byref(cfg), C.byref(wl), C.byref(fp), C.byref(h)) == 0, L.paxisim_last_error()
assert L.paxisim_dbg_enable(h) == 0
if warm:
    L.paxisim_step(h, warm)
nb = (clusters + 63) // 64
buf = (C.c_ulonglong * (nb * 16 * 16))()
L.paxisim_dbg_read(h, buf)
L.paxisim_step(h, steps)
L.paxisim_dbg_read(h, buf)
for r in range(5):
    tot = [0] * 12
    for b in range(nb):
        # dbg is indexed by replica
        for k in range(12):
            tot[k] += buf[(b * 16 + r) * 16 + k]
    st = max(1, tot[5])
    print(f"replica {r}: per wave-step setup {tot[0]/st:8.0f} loop {tot[1]/st:8.0f} barrier {tot[2]/st:8.0f} cyc;"
          f" lane-0 trips {tot[3]/st:5.2f}, records/lane {tot[4]/st/64:5.2f};"
          f" per lane-0 trip: pick+prefetch {tot[6]/max(1,tot[3]):6.0f} dispatch {tot[7]/max(1,tot[3]):6.0f}"
          f" head {tot[8]/max(1,tot[3]):6.0f} flush {tot[9]/max(1,tot[3]):6.0f}"
          f" rest {(tot[1]-tot[6]-tot[7]-tot[8]-tot[9]-tot[10]-tot[11])/max(1,tot[3]):6.0f};"
          f" per step: stage {tot[10]/st:7.0f} after lane 0 done (other lanes trips) {tot[11]/st:7.0f}")
