"""Diagnostic: workgroup residency per CU (PXS_STAMPS build).  usage: residency.py <clusters>"""
import collections
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
clusters = int(sys.argv[1])
cfg = abi.make_config(npz=[5], clusters=clusters, seed=42, window=int(os.environ.get("W", "16")), mbox_cap=16, max_delay=4, steps_per_launch=50)
wl = abi.make_workload(outstanding=8, target=0)
fp = abi.make_fault_process(drop_ppm=1000, drop_len=50, slow_ppm=1000, slow_len=50, slow_min=1, slow_max=4)
h = C.c_void_p()
assert L.paxisim_create(C.byref(cfg), C.byref(wl), C.byref(fp), C.byref(h)) == 0
assert L.paxisim_dbg_enable(h) == 0
L.paxisim_step(h, 100)
nb = (clusters + 63) // 64
buf = (C.c_ulonglong * (nb * 16 * 16))()
L.paxisim_dbg_read(h, buf)
L.paxisim_step(h, 50)
L.paxisim_dbg_read(h, buf)
rows = []
for b in range(nb):
    for r in range(5):
        d = [buf[(b * 16 + r) * 16 + k] for k in range(16)]
        if d[12]:
            hw, xcc = d[14], d[15]
            cu = (xcc & 0xF, (hw >> 13) & 3, (hw >> 12) & 1, (hw >> 8) & 0xF)
            rows.append((b, r, d[12], d[13], cu, (hw >> 4) & 3))
t0 = min(r[2] for r in rows)
per_cu = collections.defaultdict(list)
for b, r, s, e, cu, simd in rows:
    if r == 0:
        per_cu[cu].append((s - t0, e - t0, b))
print("blocks", nb, "distinct CUs", len(per_cu))
for cu, v in list(per_cu.items())[:6]:
    print(cu, sorted(v))
simds = collections.Counter((b, simd) for b, r, s, e, cu, simd in rows)
print("waves per (block, simd) histogram", collections.Counter(simds.values()))
