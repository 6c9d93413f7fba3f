"""Per-launch kernel time and delivered messages over a long config-2 run,
with a pause, to tell simulation-state effects from clock/power effects.
Usage: python tools/launch_trace.py [clusters] [launches] [pause_s]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paxi_amd import abi  # noqa: E402
from paxi_amd.sim import Simulation  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 19
L = int(sys.argv[2]) if len(sys.argv) > 2 else 30
pause = float(sys.argv[3]) if len(sys.argv) > 3 else 3.0
cfg = abi.make_config(npz=[5], clusters=C, seed=42, window=16, mbox_cap=16, max_delay=4, steps_per_launch=50)
wl = abi.make_workload(outstanding=8, target=0)
fp = abi.make_fault_process(drop_ppm=1000, drop_len=50, slow_ppm=1000, slow_len=50, slow_min=1, slow_max=4)
sim = Simulation(cfg, wl, fp)
prev = sim.stats().as_dict()
for i in range(L + 5):
    if i == L:
        time.sleep(pause)
    sim.kernel_time(reset=True)
    sim.step(50)
    sim.sync()
    ms, _ = sim.kernel_time()
    st = sim.stats().as_dict()
    d = st["delivered_total"] - prev["delivered_total"]
    fl = st["flagged"]
    print(f"launch {i:3d} ms {ms:8.2f} msgs/launch/cluster {d / C:7.1f} ns/msg/cluster-lane {ms * 1e6 / d * C / 1e6:.4f} "
          f"commits {(st['commits'] - prev['commits']) / C:6.1f} flags {fl[:6]}", flush=True)
    prev = st
sim.close()
