"""Two-mode run-to-run variance probe: back-to-back bench
processes on one box alternate between two step-kernel speeds (config 3:
23.8 / 25.6 ms per launch; config 2: 37.4 / 38.4 ms).  This creates, times
and frees the bench's simulation several times in ONE process - with the
arena allocated plainly, after a freed dummy allocation, and while a dummy
allocation is held - to see whether the mode follows where the arena lands.

  python tools/mode_probe.py <config> <rounds>
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    cfg_id = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    import torch
    from paxi_amd.sim import Simulation
    torch.cuda.set_device(0)
    d = bench.DEFAULTS[cfg_id]
    args = argparse.Namespace(window=d["window"], mbox=d["mbox"], history=512, kv=1, fz=1, crash_step=5 * d["sim_steps"])
    out = []
    held = None
    for k in range(rounds):
        mode = ["plain", "after_free", "held"][k % 3]
        if mode == "after_free":
            x = torch.empty(64 << 30, dtype=torch.uint8, device="cuda")
            del x
            torch.cuda.empty_cache()
        if mode == "held":
            held = torch.empty(64 << 30, dtype=torch.uint8, device="cuda")
        cfg, wl, fp, faults, _ = bench.workload(cfg_id, d["clusters"], 0, 0, args)
        sim = Simulation(cfg, wl, fp, faults)
        for _ in range(5):
            sim.step(d["sim_steps"])
        sim.sync()
        sim.kernel_time(reset=True)
        t0 = time.perf_counter()
        for _ in range(10):
            sim.step(d["sim_steps"])
        sim.sync()
        dt = time.perf_counter() - t0
        kms, n = sim.kernel_time()
        sim.close()
        held = None
        torch.cuda.empty_cache()
        rec = {"round": k, "mode": mode, "launch_ms": kms / max(1, n), "wall_s": dt}
        out.append(rec)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
