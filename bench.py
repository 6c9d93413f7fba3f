"""Headline benchmark (BASELINE.json): simulated messages delivered/s and
committed slots/s for 1M Multi-Paxos clusters of 5 replicas with Drop/Slow
fault injection (BASELINE config 2), on 1..8 GPUs.

One bench "step" = one pass of the hot path over the whole batch = one kernel
launch advancing every cluster of every rank by --sim-steps virtual steps.
Inputs (cluster state, mailboxes) are resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Multi-GPU: clusters are independent, so each rank owns a contiguous global
cluster range (PRNG keyed by the global id) and there is no data-path
collective; RCCL only all-reduces the statistics and the max time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

# Algorithmic bytes per delivered message: message record
# written by the sender + read by the receiver, plus the handler's state
# read-modify-write.  Phase-1 / request / reply records are priced as a
# record write + read (64 B); P1b payload entries are not counted.
ALG_BYTES = {"P2a": 160, "P2b": 144, "P3": 192, "P1a": 64, "P1b": 64, "Request": 64, "Reply": 64}
ALG_BYTES_PER_COMMIT = 64   # leader-side P2a() entry creation


def alg_bytes(delta):
    b = sum(ALG_BYTES.get(k, 64) * v for k, v in delta["delivered"].items())
    return b + ALG_BYTES_PER_COMMIT * delta["commits"]


def stats_delta(a, b):
    d = {k: b[k] - a[k] for k in ("delivered_total", "commits", "replies", "dropped", "client_requests")}
    d["delivered"] = {k: b["delivered"].get(k, 0) - a["delivered"].get(k, 0) for k in b["delivered"]}
    return d


def config2(args, rank, world, device):
    from paxi_amd import abi
    per = args.clusters
    cfg = abi.make_config(npz=[5], clusters=per, cluster_base=rank * per, seed=42, window=args.window,
                          mbox_cap=args.mbox, max_delay=4, steps_per_launch=args.sim_steps, device=device)
    wl = abi.make_workload(outstanding=8, target=0)
    fp = abi.make_fault_process(drop_ppm=1000, drop_len=50, slow_ppm=1000, slow_len=50, slow_min=1, slow_max=4)
    return cfg, wl, fp


def cpu_baseline(args):
    """The C oracle (same delivery schedule) on a bounded sample of config 2."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from paxi_amd import abi
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    clusters = args.cpu_clusters
    cfg = abi.make_config(npz=[5], clusters=clusters, seed=42, window=args.window, mbox_cap=args.mbox, max_delay=4)
    wl = abi.make_workload(outstanding=8, target=0)
    fp = abi.make_fault_process(drop_ppm=1000, drop_len=50, slow_ppm=1000, slow_len=50, slow_min=1, slow_max=4)
    out = {}
    for nthr in (1, threads):
        o = oracle_lib.OracleSim(cfg, wl, fp)
        o.step(args.warmup * args.sim_steps, threads=nthr)     # same warm-up as the GPU leg
        s0 = o.stats().as_dict()
        t0 = time.perf_counter()
        o.step(args.cpu_steps, threads=nthr)
        dt = time.perf_counter() - t0
        s1 = o.stats().as_dict()
        out[nthr] = ((s1["delivered_total"] - s0["delivered_total"]) / dt, (s1["commits"] - s0["commits"]) / dt, dt)
        o.close()
    v, c, dt = out[threads]
    v1, _, dt1 = out[1]
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": v, "unit": "messages/s", "cores": threads, "kind": "port",
            "commits_per_s": c,
            "single_thread_value": v1,
            "sample": (f"C oracle (oracle/oracle.c), config 2 on {clusters} clusters x {args.cpu_steps} steps after "
                       f"{args.warmup * args.sim_steps} warm-up steps; {threads} threads {dt:.1f}s, 1 thread "
                       f"{dt1:.1f}s ({v1:.3g} msg/s); CPU {cpu}; GOMAXPROCS n/a (no Go toolchain)")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--clusters", type=int, default=1 << 20, help="clusters per GPU")
    ap.add_argument("--sim-steps", type=int, default=50, help="virtual steps per bench step (per launch)")
    ap.add_argument("--window", type=int, default=16)
    ap.add_argument("--mbox", type=int, default=16)
    ap.add_argument("--cpu-clusters", type=int, default=16384)
    ap.add_argument("--cpu-steps", type=int, default=1600)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from paxi_amd.sim import Simulation

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if world > 1:
            dist.barrier()

    cfg, wl, fp = config2(args, rank, world, local)
    sim = Simulation(cfg, wl, fp)
    for _ in range(args.warmup):
        sim.step(args.sim_steps)
    sim.sync()
    s0 = sim.stats().as_dict()
    sim.kernel_time(reset=True)

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sim.step(args.sim_steps)
    sim.sync()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    kms, launches = sim.kernel_time()
    s1 = sim.stats().as_dict()
    d = stats_delta(s0, s1)
    violations = sim.check()

    # whole-job aggregates over RCCL: sum of work, max of time
    vec = torch.tensor([d["delivered_total"], d["commits"], alg_bytes(d), violations,
                        s1["flagged"][4], s1["flagged"][5]], dtype=torch.float64, device="cuda")
    tmax = torch.tensor([dt, kms], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(vec, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    msgs, commits, abytes, viol, unfaithful, poison = vec.tolist()
    dt_max, kms_max = tmax.tolist()

    if rank == 0:
        avg_launch_ms = kms / max(1, launches)
        achieved = alg_bytes(d) / max(1, launches) / (avg_launch_ms / 1e3) / 1e9   # rank-0 kernel, GB/s
        out = {
            "metric": "sim messages delivered/sec + committed slots/sec, 1M Paxos clusters, 1-8 GPU",
            "value": msgs / dt_max,
            "unit": "messages/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded closed-loop workload, PRNG-keyed faults)",
            "config": {"workload": "BASELINE config 2: Multi-Paxos 5 replicas x 1M clusters/GPU, Drop/Slow faults",
                       "clusters_per_gpu": args.clusters, "replicas": 5, "outstanding": 8,
                       "sim_steps_per_step": args.sim_steps, "window": args.window, "mbox_cap": args.mbox,
                       "drop": "p=1e-3/step/link, 50-step windows", "slow": "p=1e-3/step/link, 1-4 steps, 50-step windows",
                       "parallelism": f"cluster-sharded x{world}"},
            "commits_per_s": commits / dt_max,
            "sim_steps_per_s": args.sim_steps * args.steps / dt_max,
            "agreement_violations": int(viol),
            "unfaithful_clusters": int(unfaithful),
            "poisoned_clusters": int(poison),
            "kernel_ms_per_step": kms_max / args.steps,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "paxos_steps<5>", "avg_launch_ms": avg_launch_ms,
                         "alg_bytes_per_launch": alg_bytes(d) / max(1, launches)},
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    sim.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
