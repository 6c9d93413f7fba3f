"""Headline benchmark (BASELINE.json): simulated messages delivered/s and
committed slots/s, 1M Multi-Paxos clusters of 5 replicas with Drop/Slow fault
injection per GPU (BASELINE config 2), on 1..8 GPUs.

One bench "step" = one pass of the hot path over the whole batch: every
cluster of every rank advances --sim-steps virtual steps (config 2: 400, as
chunks of 20 steps, three per pipelined launch between compactions).  With the driver's --warmup 5 --steps 20 the
timed region is config 2's virtual steps 2,000-10,000: past the ~1,200-step
ramp while clusters desynchronise, and ending at the config's 10,000 steps.
Inputs (cluster state, mailboxes) are resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W] [--config 2|3|4|5]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

--config 3 (ABD + linearizability scan), 4 (FGrid 3x3, leader crash at the
first timed step, re-election at zone 2) and 5 (WPaxos) print their own lines.
Multi-GPU: see paxi_amd/dist.py — clusters shard by range, no data-path
collective; RCCL all-reduces the statistics and the max time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

# Algorithmic bytes per delivered message: the record written by
# the sender + read by the receiver, plus the handler's state read-modify-write.
# Multi-Paxos: P2a 160, P2b 144, P3 192 (+64 per committed slot for the leader's
# P2a() entry); phase-1 / request / reply records priced as a write + read (64).
# ABD: Get 80, GetReply 144, Set 96, SetReply 128 (+64 per op for the coordinator).
ALG_BYTES = {"P2a": 160, "P2b": 144, "P3": 192, "P1a": 64, "P1b": 64, "Request": 64, "Reply": 64,
             "Get": 80, "GetReply": 144, "Set": 96, "SetReply": 128, "LeaderChange": 64}
ALG_BYTES_PER_COMMIT = 64

METRIC = "sim messages delivered/sec + committed slots/sec, 1M Paxos clusters, 1-8 GPU"
FLAG_NAMES = ("WOVF", "GHOST", "MBOX_OVF", "PEND_OVF", "UNFAITHFUL", "POISON", "BALLOT_OVF", "HIST_OVF")

# per-config defaults: clusters per GPU, virtual steps per bench step, window, mailbox capacity
DEFAULTS = {1: dict(clusters=1, sim_steps=3010, window=32, mbox=16),
            2: dict(clusters=1 << 20, sim_steps=400, window=16, mbox=32),
            3: dict(clusters=1 << 20, sim_steps=80, window=16, mbox=16),
            4: dict(clusters=1 << 19, sim_steps=200, window=16, mbox=24),
            5: dict(clusters=1 << 18, sim_steps=200, window=8, mbox=24)}
# Config 5 runs at window 8 (round 6): it never reaches the bound at 8 or 16 (WOVF 0 in both), its per-type
# counts, flags and shard digests are equal at both windows on the GPU (profiles/r6/g1), and the oracle's
# states and instances equal W = 64's (tests/test_bounded_model.py); at 8 an instance and its window share
# one co-located block
# virtual steps per chunk: 50 (configs 4 and 5 are best at 50, A/B r5aa);
# config 2 20, compacted every 3 chunks (DESIGN.md §5.9, A/Bs r5x, r5aa: 25-step
# chunks every 75 +0.9 / +2.2% over 50-step chunks every 100, 20-step chunks
# every 60 another +0.8%); config 3 20: its 80-step
# bench step is one pipelined launch of 4 chunks (A/B r5v: +5.7% against one
# 80-step launch, itself +2.7% over 50-step launches in round 4);
# PAXISIM_LAUNCH_STEPS overrides.  The library fuses up to 4 chunks per launch
# (PAXISIM_PIPE)
LAUNCH_DEFAULT = {2: 20, 3: 20}


def launch_steps(cfg_id):
    env = os.environ.get("PAXISIM_LAUNCH_STEPS")
    return int(env) if env else LAUNCH_DEFAULT.get(cfg_id, 50)


def alg_bytes(delta):
    b = sum(ALG_BYTES.get(k, 64) * v for k, v in delta["delivered"].items())
    return b + ALG_BYTES_PER_COMMIT * delta["commits"]


def stats_delta(a, b):
    d = {k: b[k] - a[k] for k in ("delivered_total", "commits", "replies", "dropped", "client_requests")}
    d["delivered"] = {k: b["delivered"].get(k, 0) - a["delivered"].get(k, 0) for k in b["delivered"]}
    return d


def build_id():
    """The source fingerprint compiled into the loaded libpaxisim.so
    (paxisim_build_id): the binary this run measured, not the tree beside it."""
    from paxi_amd import sim as psim
    return psim.build_id()


def source_id():
    """Fingerprint of the HIP sources in this tree (what build() would compile)."""
    import __graft_entry__ as ge
    return ge.source_id()


def workload(cfg_id, clusters, base, device, args):
    """(cfg, workload, fault process, scripted faults, description) of a BASELINE config."""
    from paxi_amd import abi
    if cfg_id == 1:
        # the reference's own CPU case (bin/simulation.sh): 3 replicas, one
        # client, 1000 sequential writes to 1.1, no faults; 3 steps a request
        cfg = abi.make_config(npz=[3], clusters=clusters, cluster_base=base, seed=1, window=args.window,
                              mbox_cap=args.mbox, max_delay=0, steps_per_launch=launch_steps(cfg_id), device=device,
                              kv=args.kv)
        wl = abi.make_workload(outstanding=1, max_requests=1000, target=[0])
        return cfg, wl, None, [], {
            "workload": "BASELINE config 1: Multi-Paxos 3 replicas, 1 client, 1000 writes, no faults "
                        "(the reference's CPU case; run with --warmup 0 --steps 1)", "replicas": 3, "outstanding": 1}
    if cfg_id == 2:
        cfg = abi.make_config(npz=[5], clusters=clusters, cluster_base=base, seed=42, window=args.window,
                              mbox_cap=args.mbox, max_delay=4, steps_per_launch=launch_steps(cfg_id), device=device,
                              kv=args.kv)
        wl = abi.make_workload(outstanding=8, target=0)
        fp = abi.make_fault_process(drop_ppm=1000, drop_len=50, slow_ppm=1000, slow_len=50, slow_min=1, slow_max=4)
        return cfg, wl, fp, [], {
            "workload": "BASELINE config 2: Multi-Paxos 5 replicas x 1M clusters/GPU, Drop/Slow faults",
            "replicas": 5, "outstanding": 8, "drop": "p=1e-3/step/link, 50-step windows",
            "slow": "p=1e-3/step/link, 1-4 steps, 50-step windows"}
    if cfg_id == 3:
        cfg = abi.make_config(protocol=abi.ABD, npz=[5], clusters=clusters, cluster_base=base, seed=42, keys=16,
                              mbox_cap=args.mbox, max_delay=4, steps_per_launch=launch_steps(cfg_id), device=device,
                              history=args.history)
        wl = abi.make_workload(outstanding=4, target=[0, 1, 2, 3], write_ppm=500_000)
        return cfg, wl, None, [], {
            "workload": "BASELINE config 3: ABD 5 replicas x 1M clusters/GPU, 16 keys, 50% writes, "
                        "linearizability scan on device", "replicas": 5, "outstanding": 4}
    if cfg_id == 4:
        # Clients talk to leader 1.1 (replica 0) until it crashes for good at
        # crash_step; from then on a second set of clients talks to 2.1
        # (replica 3), whose first request runs phase 1 under -ephemeral_leader
        # (paxos/replica.go:61) and re-elects it.  The first set stays blocked on
        # the crashed leader: Paxi's HTTP client has no retry.
        # --fz 1: FGridQ1/Q2(1) (quorum.go:99-119); --fz 0: the Grid variant,
        # GridRow/GridColumn (quorum.go:85-97), Q1 = Q2 = 3 replicas at 3x3
        c = args.crash_step
        fz = getattr(args, "fz", 1)
        q1, q2 = (abi.Q_FGRID_Q1, abi.Q_FGRID_Q2) if fz else (abi.Q_GRID_ROW, abi.Q_GRID_COLUMN)
        cfg = abi.make_config(npz=[3, 3, 3], clusters=clusters, cluster_base=base, seed=42, q1=q1,
                              q2=q2, fz=fz, ephemeral_leader=1, window=args.window, mbox_cap=args.mbox,
                              max_delay=0, steps_per_launch=launch_steps(cfg_id), device=device,
                              kv=args.kv)
        wl = abi.make_workload(outstanding=8, target=[0, 0, 0, 0, 3, 3, 3, 3], start_step=[0, 0, 0, 0, c, c, c, c])
        faults = [abi.make_fault(abi.FAULT_CRASH, 0, step_from=c)]
        return cfg, wl, None, faults, {
            "workload": (f"BASELINE config 4: FGrid 3x3 (fz={fz})" if fz else
                         "BASELINE config 4, Grid variant: 3x3 GridRow/GridColumn (fz=0)") +
                        f" x 512K clusters/GPU; leader 1.1 crashes for good at "
                        f"step {c}, clients then turn to 2.1 which re-elects itself (ephemeral leader)",
            "replicas": 9, "outstanding": "4 -> 1.1 from step 0, 4 -> 2.1 from the crash", "crash_step": c,
            "fz": fz}
    if cfg_id == 5:
        cfg = abi.make_config(protocol=abi.WPAXOS, npz=[3, 3, 3], keys=8, fz=0, adaptive=1, policy_threshold=3,
                              clusters=clusters, cluster_base=base, seed=42, window=args.window, mbox_cap=args.mbox,
                              max_delay=0, steps_per_launch=launch_steps(cfg_id), device=device,
                              kv=args.kv)
        wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000)
        return cfg, wl, None, [], {
            "workload": "BASELINE config 5: WPaxos 3 zones x 3 nodes, 8 keys (kpaxos instances) per cluster, "
                        "Grid Q1/Q2, consecutive policy (threshold 3) object stealing, 70% zone-local keys",
            "replicas": 9, "keys": 8, "outstanding": 9}
    raise SystemExit(f"unknown config {cfg_id}")


def measured_traffic(args, kernel, mbox, bid, alg_per_launch=None):
    """HBM bytes per launch from the PMC passes of tools/traffic.sh (committed as
    profiles/traffic_config<c>.json), attached when the record was measured on
    this build (source fingerprint) and this workload (kernel, clusters, window,
    mailbox, launch size) over this bench window (warmup, steps): the
    simulation is seeded, so a launch at a given simulated step moves the same
    bytes in every run, but bytes per launch change along the run (a ~1,200-step
    ramp, then clusters dying), so a record of another window is not attached.
    Counters cannot be read from inside this process."""
    fz0 = args.config == 4 and getattr(args, "fz", 1) == 0          # the Grid variant has its own record
    path = os.path.join(ROOT, "profiles", f"traffic_config{args.config}{'_fz0' if fz0 else ''}.json")
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None
    same = (t.get("kernel") == kernel and t.get("clusters_per_gpu") == args.clusters
            and t.get("sim_steps_per_step") == args.sim_steps and t.get("window") == args.window
            and t.get("mbox_cap") == mbox and t.get("build_id") == bid
            and t.get("warmup") == args.warmup and t.get("steps") == args.steps
            and (args.config != 4 or t.get("fz", 1) == getattr(args, "fz", 1)))
    # the same launch structure (chunk length, chunks per launch): the seeded run's algorithmic
    # bytes per launch are then identical
    if same and alg_per_launch is not None and t.get("alg_bytes_per_launch"):
        same = abs(t["alg_bytes_per_launch"] - alg_per_launch) <= 1e-9 * alg_per_launch
    if not same:
        return None
    return {"bytes_per_launch": t["bytes_per_launch"], "source": os.path.relpath(path, ROOT),
            "window": {"warmup": t.get("warmup"), "steps": t.get("steps")}}


def cpu_threads():
    """Host threads for the CPU baseline: the CPUs this process may run on
    (sched_getaffinity), capped by a cgroup CPU quota when one is set;
    PAXISIM_CPU_THREADS overrides."""
    if os.environ.get("PAXISIM_CPU_THREADS"):
        return int(os.environ["PAXISIM_CPU_THREADS"]), "PAXISIM_CPU_THREADS"
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    why = f"sched_getaffinity ({n} of os.cpu_count() {os.cpu_count()})"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            q = max(1, int(int(quota) / int(period)))
            if q < n:
                n, why = q, f"cgroup cpu.max quota {quota}/{period}"
    except (OSError, ValueError):
        pass
    return n, why


def host_physical_cores():
    """Physical cores of the host (sockets x cores per socket), from sysfs topology."""
    try:
        ids = set()
        base = "/sys/devices/system/cpu"
        for d in os.listdir(base):
            if d.startswith("cpu") and d[3:].isdigit():
                t = os.path.join(base, d, "topology")
                ids.add((open(os.path.join(t, "physical_package_id")).read().strip(),
                         open(os.path.join(t, "core_id")).read().strip()))
        return len(ids) or None
    except OSError:
        return None


def cpu_baseline(args, sim=None, min_s=3.0):
    """The C oracle (same delivery schedule) over exactly the GPU leg's timed
    window of virtual steps, after the same warm-up: one thread on 256
    clusters, then all usable host threads on enough clusters for >= min_s
    seconds (the rate changes along a run, so the window must match).

    The oracle is the checker too: its samples end at the step the GPU handle
    `sim` (rank 0: global clusters from 0) ended at, so the replica states of
    those clusters must be equal; a second sample reruns random, WOVF- and
    GHOST-flagged and frozen GPU clusters one by one (tests/parity_sample.py).
    Both go into res["parity_sampled"]."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    threads, why = cpu_threads()
    warm, window = args.warmup * args.sim_steps, args.steps * args.sim_steps
    out = {}
    checked = {"clusters": 0, "equal": 0}

    def sample(nthr, clusters):
        cfg, wl, fp, faults, _ = workload(args.config, clusters, 0, 0, args)
        o = oracle_lib.OracleSim(cfg, wl, fp, faults)
        o.step(warm, threads=nthr)
        s0 = o.stats().as_dict()
        t0 = time.perf_counter()
        o.step(window, threads=nthr)
        dt = time.perf_counter() - t0
        s1 = o.stats().as_dict()
        if sim is not None:   # the checker: the same clusters on the GPU, at the same step
            n = min(clusters, sim.cfg.clusters)
            N = sim.N
            a, b = sim.read_state(0, n), o.read_state(0, n)
            eq = sum(1 for c in range(n) if all(a[c * N + r].as_tuple() == b[c * N + r].as_tuple()
                                                for r in range(N)))
            checked["clusters"] = max(checked["clusters"], n)
            checked["equal"] = eq if n == checked["clusters"] else checked["equal"]
        o.close()
        return ((s1["delivered_total"] - s0["delivered_total"]) / dt, (s1["commits"] - s0["commits"]) / dt,
                dt, clusters)

    out[1] = sample(1, 256)
    if out[1][2] < 2.0:   # a single-thread sample of >= 2 s
        out[1] = sample(1, int(256 * 2.2 / max(out[1][2], 1e-3)))
    if threads > 1:       # the multi-thread sample sized for >= min_s seconds
        dt1, cl1 = out[1][2], out[1][3]
        out[threads] = sample(threads, int(cl1 * threads * max(1.0, min_s / max(dt1, 1e-3))))
    v, c, dt, cl = out[threads]
    v1, _, dt1, cl1 = out[1]
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    phys = host_physical_cores()
    res = {"value": v, "unit": "messages/s", "cores": threads, "kind": "port", "commits_per_s": c,
           "single_thread_value": v1, "host_cpus": os.cpu_count(), "host_physical_cores": phys,
           "threads_from": why,
           "sample": (f"C oracle (oracle/oracle.c), config {args.config}, virtual steps [{warm}, {warm + window}) "
                      f"after the same warm-up as the GPU leg: {threads} threads on {cl} clusters ({dt:.1f}s), "
                      f"1 thread on {cl1} clusters ({dt1:.1f}s, {v1:.3g} msg/s); CPU {cpu}; "
                      f"GOMAXPROCS n/a (no Go toolchain)")}
    if phys and phys > threads:
        # not measured: this process may use only `threads` CPUs of the host
        res["linear_estimate_all_physical_cores"] = v / threads * phys
    if sim is not None:
        import parity_sample
        cfg, wl, fp, faults, _ = workload(args.config, sim.cfg.clusters, 0, 0, args)
        picks = parity_sample.choose(sim, n_random=64, n_flag=32, n_frozen=32)
        pr = parity_sample.check(sim, cfg, wl, fp, faults, warm + window, picks, threads=threads)
        k = checked["clusters"] + pr["compared"]
        eq = checked["equal"] + pr["equal"]
        res["parity_sampled"] = f"{eq}/{k}"
        res["parity_detail"] = {"contiguous_clusters": [0, checked["clusters"]], "contiguous_equal": checked["equal"],
                                "picked": pr["by_kind"], "picked_equal": pr["equal"],
                                "mismatches": pr["mismatches"], "at_step": warm + window,
                                "compared": "every replica's paxisim_read_state record (+ instances / history)"}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5])
    ap.add_argument("--clusters", type=int, default=None, help="clusters per GPU (default: the config's)")
    ap.add_argument("--sim-steps", type=int, default=None, help="virtual steps per bench step")
    ap.add_argument("--window", type=int, default=None)
    ap.add_argument("--mbox", type=int, default=None)
    ap.add_argument("--history", type=int, default=512, help="config 3: ops recorded per replica")
    ap.add_argument("--fz", type=int, default=1, choices=[0, 1],
                    help="config 4: FGrid fz (1) or the Grid variant GridRow/GridColumn (0)")
    ap.add_argument("--crash-step", type=int, default=None,
                    help="config 4: step of the leader crash (default: the first timed step)")
    ap.add_argument("--kv", type=int, default=1, choices=[0, 1],
                    help="replicas execute into a Database (db.go Execute) - the reference always does")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-shard-check", action="store_true",
                    help="skip the per-rank state digests (sharding invariance, SURVEY 8e)")
    args = ap.parse_args()
    for k, v in DEFAULTS[args.config].items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    if args.crash_step is None:
        args.crash_step = args.warmup * args.sim_steps

    import torch
    import torch.distributed as dist
    from paxi_amd import abi
    from paxi_amd import dist as pdist
    from paxi_amd.sim import Simulation

    rank, world, local = pdist.env_rank()
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # PAXISIM_DIST_BACKEND=gloo rehearses the N>1 flow with several ranks on
    # one GPU (RCCL refuses two ranks on one device); the default is RCCL.
    backend = os.environ.get("PAXISIM_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    def barrier():
        if world > 1:
            dist.barrier()

    base, count = pdist.shard(args.clusters, rank)
    cfg, wl, fp, faults, desc = workload(args.config, count, base, local, args)
    sim = Simulation(cfg, wl, fp, faults)
    pd = None
    if world > 1 and backend == "nccl":
        # the statistics go through the library's own RCCL communicator
        # (paxisim_dist_init_rank); torch.distributed only ships its id
        from paxi_amd.sim import Dist
        uid = [Dist.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        pd = Dist.join(sim, uid[0], world, rank)
    for _ in range(args.warmup):
        sim.step(args.sim_steps)
    sim.sync()
    s0 = sim.stats().as_dict()
    active_start = sim.active_clusters()
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
    lin = None
    if args.config == 3:
        tl = time.perf_counter()
        a, n, skipped = sim.linearizable()
        lin = {"anomalies": a, "ops_checked": n, "partitions_skipped": skipped, "scan_s": time.perf_counter() - tl}

    # sharding invariance: every rank digests the states of its
    # local clusters [C/2, C/2+256); at N=1 the same global ranges of ranks
    # 1..7 are simulated by small handles of their own, so the N=8 run's rank-g
    # digest must equal the N=1 run's "virtual" rank-g digest
    shard_digests = None
    if not args.no_shard_check:
        dlo, dn = pdist.digest_range(args.clusters)
        mine = pdist.state_digest(sim, dlo, dn)
        got = pdist.gather_digests(mine, world)
        if world == 1:
            for g in range(1, 8):
                c2, w2, f2, x2, _ = workload(args.config, dn, g * args.clusters + dlo, local, args)
                s2 = Simulation(c2, w2, f2, x2)
                s2.step((args.warmup + args.steps) * args.sim_steps)
                got[g] = pdist.state_digest(s2, 0, dn)
                s2.close()
        shard_digests = {"clusters_per_rank": [dlo, dlo + dn], "digests": {str(k): v for k, v in got.items()},
                         "virtual": world == 1}

    st1 = sim.stats()
    vals = pdist.stats_counters(d, alg_bytes(d), violations, s1["flagged"], agree_compared=st1.agree_compared,
                                agree_missed=st1.agree_missed, active=sim.active_clusters(),
                                active_start=active_start)
    if pd is not None:
        tot, (dt_max, kms_max) = pdist.reduce_counters_abi(pd, vals, [dt, kms])
    else:
        tot, (dt_max, kms_max) = pdist.reduce_counters(vals, [dt, kms], device="cuda" if backend == "nccl" else "cpu")

    if rank == 0:
        avg_launch_ms = kms / max(1, launches)
        achieved = alg_bytes(d) / max(1, launches) / (avg_launch_ms / 1e3) / 1e9   # rank 0's kernel, GB/s
        # config 5: instance scalars in the packed HBM table (WPaxosProto), or with PAXISIM_WLDS=1 in the tile image
        wp = "WPaxosProtoL" if os.environ.get("PAXISIM_WLDS", "0") != "0" else "WPaxosProto"
        proto = {3: "AbdProto", 5: wp}.get(args.config, "PaxosProto")
        # the library's default step kernel is the serial one
        kname = "sim_steps" if os.environ.get("PAXISIM_SERIAL") == "0" else "sim_serial"
        if kname == "sim_serial" and args.steps * args.sim_steps > launches * launch_steps(args.config):
            kname = "sim_serial_pipe"             # chunks fused into pipelined launches
        occ = sim.occupancy()
        desc.update({"tiles_per_cu": occ[0], "lds_per_tile": occ[1], "staged_msgs": occ[2]})
        desc.update({"clusters_per_gpu": args.clusters, "sim_steps_per_step": args.sim_steps,
                     "timed_sim_steps": [args.warmup * args.sim_steps, (args.warmup + args.steps) * args.sim_steps],
                     "window": args.window, "mbox_cap": cfg.mbox_cap, "parallelism": f"cluster-sharded x{world}",
                     "database": "kv (db.go Execute per replica)" if cfg.kv or args.config == 3 else "off"})
        bid = build_id()
        out = {
            "metric": METRIC,
            "value": tot["delivered_total"] / dt_max,
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
            "config": desc,
            "commits_per_s": tot["commits"] / dt_max,
            # rank 0's timed-window deliveries by message type (a W=16 / W=64 line pair must agree)
            "delivered_by_type_rank0": {k: int(v) for k, v in d["delivered"].items() if v},
            "sim_steps_per_s": args.sim_steps * args.steps / dt_max,
            "agreement_violations": int(tot["violations"]),
            "agreement_coverage": {"checkpoints_compared": int(tot["agree_compared"]),
                                   "checkpoints_missed": int(tot["agree_missed"]),
                                   "every": "16 executed slots, against the first executor (paxisim_check)"},
            "active_clusters_start": int(tot["active_start"]),
            "active_clusters_end": int(tot["active"]),
            # the live set shrinks over the window (no-retry semantics): the rate per
            # live cluster (mean of the window's start and end counts) compares runs across that decay
            "msgs_per_s_per_live_cluster": tot["delivered_total"] / dt_max /
                                           max(1.0, 0.5 * (tot["active_start"] + tot["active"])),
            "unfaithful_clusters": int(tot["flag_UNFAITHFUL"]),
            "poisoned_clusters": int(tot["flag_POISON"]),
            "flagged_clusters": {n: int(tot["flag_" + n]) for n in FLAG_NAMES},
            "clusters_total": args.clusters * world,
            "kernel_ms_per_step": kms_max / args.steps,
            # where a bench step's wall time goes: the step kernel (HIP events on its stream) and the
            # rest - compaction and phase binning, the statistics, launch gaps; per virtual step a
            # wave's replica-steps are a chain of dependent HBM round trips (config 1: one wave)
            "time_split": {"kernel_ms_per_step": kms / args.steps,
                           "other_ms_per_step": max(0.0, dt - kms / 1e3) / args.steps * 1e3,
                           "us_per_virtual_step": dt / (args.steps * args.sim_steps) * 1e6,
                           "kernel_us_per_virtual_step": kms / (args.steps * args.sim_steps) * 1e3,
                           "msgs_per_virtual_step": tot["delivered_total"] / (args.steps * args.sim_steps)},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": f"{kname}<{abi.n_replicas(cfg)},{proto}>",
                         "avg_launch_ms": avg_launch_ms, "launches": launches,
                         "alg_bytes_per_launch": alg_bytes(d) / max(1, launches)},
            "build_id": bid,
            "build_id_of": "the loaded libpaxisim.so (paxisim_build_id)",
            "build_matches_sources": bid == source_id(),
        }
        tr = measured_traffic(args, out["roofline"]["kernel"], cfg.mbox_cap, bid, out["roofline"]["alg_bytes_per_launch"])
        if tr is not None:
            out["roofline"]["traffic"] = tr["bytes_per_launch"]
            out["roofline"]["traffic_source"] = tr["source"]
            out["roofline"]["traffic_window"] = tr["window"]
        try:   # the achievable HBM bandwidth on this part (tools/probe/copy_bw.hip, the guide's float4 copy shape),
            # beside the spec peak; the guide's own figure is 6.29 TB/s (MI355X_MICROARCH.md:36)
            cb = json.load(open(os.path.join(ROOT, "profiles", "r6", "copy_bw.json")))
            out["roofline"]["measured_copy_peak"] = {"value": cb["copy_GBps"], "read_only": cb["read_GBps"],
                                                     "frac_of_it": achieved / cb["copy_GBps"],
                                                     "source": "profiles/r6/copy_bw.json",
                                                     "guide": "6.29 TB/s float4 copy, MI355X_MICROARCH.md:36"}
        except (OSError, ValueError, KeyError):
            pass
        if lin is not None:
            out["linearizability"] = lin
        if shard_digests is not None:
            out["shard_digests"] = shard_digests
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, sim)
            if "parity_sampled" in out["cpu_baseline"]:
                out["parity_sampled"] = out["cpu_baseline"]["parity_sampled"]
        print(json.dumps(out), flush=True)
    if pd is not None:
        pd.close()
    sim.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
