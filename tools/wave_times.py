"""Diagnostic: how well one launch of the serial step kernel fills the GPU
(PXS_WAVE_TIMES build, var/v_wavetimes.so).  Every live workgroup (one wave,
64 clusters) records its start and end on the 100 MHz clock; per launch this
prints the makespan, the busy fraction busy / (slots x makespan) with slots =
the resident waves the occupancy allows, the tail (time from the first moment
fewer than `slots` waves run until the end), and the spread of wave durations
by dispatch order.

  python tools/wave_times.py <config> <warm launches> <launches> [clusters] [chunks]

With chunks > 1 each measured call steps chunks x the chunk length, which the
library runs as pipelined launches when its build records
every (tile, chunk) item (the PXS_WAVE_TIMES pipelined variant): the busy
fraction is then over all items of the call.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from paxi_amd import abi  # noqa: E402
import bench  # noqa: E402

L = C.CDLL(os.path.join(ROOT, os.environ.get("PAXISIM_WT_LIB", "var/v_wavetimes.so")))
abi.declare(L, "paxisim")
L.paxisim_step.argtypes = [C.c_void_p, C.c_uint32]
L.paxisim_dbg_enable.argtypes = [C.c_void_p]
L.paxisim_dbg_read.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
L.paxisim_occupancy.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]


def main():
    config, warm, launches = (int(a) for a in sys.argv[1:4])
    d = bench.DEFAULTS[config]
    clusters = int(sys.argv[4]) if len(sys.argv) > 4 and int(sys.argv[4]) else d["clusters"]
    chunks = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    a = argparse.Namespace(window=d["window"], mbox=d["mbox"], history=512, kv=1, fz=1, crash_step=5 * d["sim_steps"])
    cfg, wl, fp, faults, _ = bench.workload(config, clusters, 0, 0, a)
    S = bench.LAUNCH_DEFAULT.get(config, 50)
    cfg.steps_per_launch = S
    h = C.c_void_p()
    assert L.paxisim_create(C.byref(cfg), C.byref(wl), C.byref(fp) if fp is not None else None, C.byref(h)) == 0, \
        L.paxisim_last_error()
    for f in faults:
        assert L.paxisim_fault_add(h, C.byref(f)) == 0
    assert L.paxisim_dbg_enable(h) == 0
    bpc, lds, stg = C.c_int(), C.c_uint32(), C.c_uint32()
    assert L.paxisim_occupancy(h, C.byref(bpc), C.byref(lds), C.byref(stg)) == 0
    slots = bpc.value * 256
    nb = (clusters + 63) // 64
    buf = (C.c_ulonglong * (nb * 16 * 48))()   # the library's dbg buffer: 768 words per tile
    for _ in range(warm):
        L.paxisim_step(h, S)
    L.paxisim_dbg_read(h, buf)
    out, prev = [], {}
    for k in range(launches):
        L.paxisim_step(h, S * chunks)
        L.paxisim_dbg_read(h, buf)
        if chunks > 1:                                         # every (tile, chunk) item of the call
            a = np.frombuffer(buf, dtype=np.uint64, count=2 * nb * (chunks + 1)).reshape(chunks + 1, nb, 2).astype(np.int64)
            piped = (a[1:, :, 1] > 0).any(axis=0)              # slot 0: sim_serial launches (and each tile's last item)
            t = np.concatenate([a[1:].reshape(-1, 2), a[0][~piped]])
            t = t[t[:, 1] > 0]
            dur = (t[:, 1] - t[:, 0]) / 100.0
            span = (t[:, 1].max() - t[:, 0].min()) / 100.0
            rec = {"call": warm + k, "items": int(len(t)), "slots": slots, "makespan_us": round(span, 1),
                   "busy_frac": round(float(dur.sum() / (slots * span)), 3), "item_us_mean": round(float(dur.mean()), 1)}
            out.append(rec)
            print(json.dumps(rec), flush=True)
            continue
        t = np.frombuffer(buf, dtype=np.uint64, count=2 * nb).reshape(nb, 2).astype(np.int64)
        live = t[:, 1] > 0
        t0, t1 = t[live, 0], t[live, 1]
        base = t0.min()
        span = (t1.max() - base) / 100.0                     # us
        dur = (t1 - t0) / 100.0
        busy = dur.sum() / (slots * span)
        ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t1, -np.ones_like(t1)], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        run = np.cumsum(ev[:, 1])
        full = np.nonzero(run >= min(slots, live.sum()))[0]
        tail_from = ev[full[-1], 0] if len(full) else base
        q = np.array_split(dur, 4)                             # by dispatch order (block index)
        def greedy(d):                                         # list scheduling on `slots` wave slots
            free = np.zeros(min(slots, len(d)))
            for x in d:
                i = free.argmin()
                free[i] += x
            return free.max()
        live_blk = np.nonzero(live)[0]
        order = np.argsort(t0, kind="stable")
        sim_block = greedy(dur[np.argsort(live_blk, kind="stable")])
        sim_lpt = greedy(np.sort(dur)[::-1])
        # longest-predicted-first: the previous launch's duration of the same tile as the prediction
        pred = np.array([prev.get(int(b), 0.0) for b in live_blk])
        sim_pred = greedy(dur[np.argsort(-pred, kind="stable")])
        prev.clear()
        prev.update({int(b): float(x) for b, x in zip(live_blk, dur)})
        rec = {"launch": warm + k, "waves": int(live.sum()), "slots": slots, "makespan_us": round(span, 1),
               "busy_frac": round(float(busy), 3), "tail_us": round((t1.max() - tail_from) / 100.0, 1),
               "wave_us_mean": round(float(dur.mean()), 1), "wave_us_max": round(float(dur.max()), 1),
               "wave_us_by_quarter": [round(float(x.mean()), 1) for x in q],
               "last_start_us": round((t0.max() - base) / 100.0, 1), "max_running": int(run.max()),
               "dispatch_in_block_order": bool(np.all(np.diff(live_blk[order]) > 0)),
               "model_block_order_us": round(float(sim_block), 1), "model_longest_first_us": round(float(sim_lpt), 1),
               "model_predicted_first_us": round(float(sim_pred), 1),
               "duration_corr_prev": round(float(np.corrcoef(pred, dur)[0, 1]), 3) if pred.any() else None}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    L.paxisim_destroy(h)


if __name__ == "__main__":
    main()
