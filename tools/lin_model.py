"""Instrumented Python model of the GPU linearizability checker (lin_kernel.h
LinReg.run, the reference's checker.go:69-104 / lib/graph.go:180-232) on
config-3-like ABD histories from the oracle: counts, per op, the work each
phase of run() does (adds, look-ahead steps, reach BFS levels, DFS steps),
so a redesign can be priced before it is built.  Anomaly totals are checked
against the oracle's own checker.

  python tools/lin_model.py [clusters] [steps]
"""
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from paxi_amd import abi  # noqa: E402
import oracle_lib as ol  # noqa: E402

C = collections.Counter()
SHORTCUT = os.environ.get("LIN_SHORTCUT", "1") == "1"


def run(ops):
    """ops: sorted list of [is_write, value, start, end]; returns anomalies."""
    n = len(ops)
    vid = [None] * n
    opv, vst, ven, vvl, msc = [], [], [], [], []
    rows = []            # successor bitsets, by vertex
    present = writes = 0
    st = {"nv": 0}

    def add(o):
        if vid[o] is not None:
            return
        w, val, s, e = ops[o]
        i = st["nv"]
        st["nv"] += 1
        vid[o] = i
        opv.append(o); vst.append(s); ven.append(e); vvl.append(val); rows.append(0); msc.append(1 << 40)
        nonlocal present, writes
        for v in range(i):
            if (present >> v) & 1 and ven[v] < s:
                rows[v] |= 1 << i
                msc[v] = min(msc[v], e)
        present |= 1 << i
        if w:
            writes |= 1 << i
        C["add"] += 1

    def remove(r):
        nonlocal present
        present &= ~(1 << r)
        rows[r] = 0
        for v in range(st["nv"]):
            rows[v] &= ~(1 << r)

    def match(out):
        for v in range(st["nv"]):
            if (present >> v) & 1 and (writes >> v) & 1 and vvl[v] == out:
                return v
        return None

    def merge(r, m):
        em = min(ven[m], ven[r])
        for v in range(st["nv"]):
            if v != m and (rows[v] >> r) & 1:
                rows[v] |= 1 << m
            if v != m and (rows[v] >> m) & 1:
                msc[v] = min(msc[v], em)
        if ven[r] < ven[m]:
            ven[m] = ven[r]
            ops[opv[m]][3] = ven[r]
        remove(r)

    def inverted_any():
        # an edge u -> t with u.start > t.end may exist (msc: a lower bound of the successors' ends)
        return any((present >> u) & 1 and vst[u] > msc[u] for u in range(st["nv"]))

    def reaches_self(m):
        C["reach_calls"] += 1
        R = F = 1 << m
        while True:
            C["reach_levels"] += 1
            nx = 0
            f = F
            while f:
                v = (f & -f).bit_length() - 1
                f &= f - 1
                nx |= rows[v]
            if (nx >> m) & 1:
                C["reach_true"] += 1
                return True
            nx &= present & ~R
            if not nx:
                return False
            R |= nx
            F = nx

    def x_set():
        # vertices that reach a cycle: what is left after peeling sinks (C["peel"] counts rounds)
        alive = present
        while True:
            C["peel"] += 1
            sinks = 0
            a = alive
            while a:
                v = (a & -a).bit_length() - 1
                a &= a - 1
                if not (rows[v] & alive):
                    sinks |= 1 << v
            if not sinks:
                return alive
            alive &= ~sinks

    def cycle():
        C["cycle_calls"] += 1
        X = x_set()
        black = gray = 0
        pruned = 0
        for root in range(st["nv"]):
            if not (present >> root) & 1 or (black >> root) & 1:
                continue
            stack, v, k = [], root, 0
            gray |= 1 << root
            while True:
                C["dfs_steps"] += 1
                if (X >> v) & 1:
                    C["dfs_steps_in_X"] += 1
                c = rows[v] & ~black & ~((1 << k) - 1)
                if not c:
                    gray &= ~(1 << v)
                    black |= 1 << v
                    if not stack:
                        break
                    v, k = stack.pop()
                    continue
                u = (c & -c).bit_length() - 1
                if (gray >> u) & 1:
                    return True, gray
                stack.append((v, u + 1))
                gray |= 1 << u
                v, k = u, 0
        return False, gray

    def cut(gray):
        changed = False
        g = gray
        while g:
            u = (g & -g).bit_length() - 1
            g &= g - 1
            t_ = gray
            while t_:
                t = (t_ & -t_).bit_length() - 1
                t_ &= t_ - 1
                if vst[u] > ven[t] and (rows[u] >> t) & 1:
                    rows[u] &= ~(1 << t)
                    C["cut_edges"] += 1
                    changed = True
        return changed

    maybe_cyclic = False
    anomalies = 0
    for i in range(n):
        add(i)
        if ops[i][0]:
            continue
        C["reads"] += 1
        j = i + 1
        while j < n and not (ops[i][3] < ops[j][2]) and not (ops[j][3] < ops[i][2]):
            C["look_steps"] += 1
            if ops[j][0]:
                C["look_adds_tried"] += 1
                add(j)
            j += 1
        r = vid[i]
        m = match(ops[i][1])
        if m is not None:
            C["matches"] += 1
            merge(r, m)
        cyc, gray = False, 0
        was = maybe_cyclic
        if SHORTCUT and maybe_cyclic and not inverted_any():
            # the graph stays cyclic (no edge on a cycle was removed since) and no
            # edge can be cut: Cycle() finds a cycle, cut() changes nothing
            C["shortcut"] += 1
            anomalies += 1
            continue
        if maybe_cyclic:
            C["cyc_while_cyclic"] += 1
            inv = 0
            for u in range(st["nv"]):
                if (present >> u) & 1:
                    r_ = rows[u]
                    while r_:
                        t = (r_ & -r_).bit_length() - 1
                        r_ &= r_ - 1
                        if vst[u] > ven[t]:
                            inv += 1
            C["cyclic_reads_no_inverted_edge"] += inv == 0
            cyc, gray = cycle()
        elif m is not None and reaches_self(m):
            cyc, gray = cycle()
        if cyc:
            anomalies += 1
            changed = cut(gray)
            if not changed:
                C["cut_noop" + ("_cyclic" if was else "_fresh")] += 1
            if SHORTCUT and not changed:
                maybe_cyclic = True                      # the same graph: still cyclic
            elif not was:
                maybe_cyclic = reaches_self(m)
            else:
                maybe_cyclic = cycle()[0]
        else:
            maybe_cyclic = False
    return anomalies


def main():
    clusters = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    cfg = abi.make_config(protocol=abi.ABD, npz=[5], clusters=clusters, seed=42, keys=16, mbox_cap=16, max_delay=4,
                          history=512)
    wl = abi.make_workload(outstanding=4, target=[0, 1, 2, 3], write_ppm=500_000)
    o = ol.OracleSim(cfg, wl)
    o.step(steps, threads=8)
    ref_anom, ref_ops = o.linearizable()
    total, sizes = 0, collections.Counter()
    for c in range(clusters):
        h = o.history(c)
        for k in range(16):
            part = [[w, v if w else v, s, e] for (key, w, v, s, e) in h if key == k]
            part = sorted(part, key=lambda x: x[2])          # stable: canonical order on ties
            sizes[min(len(part) // 16 * 16, 256)] += 1
            C["ops"] += len(part)
            C["partitions"] += 1
            total += run(part)
    o.close()
    out = {"clusters": clusters, "steps": steps, "anomalies_model": total, "anomalies_oracle": ref_anom,
           "ops_oracle": ref_ops, "counts": dict(C),
           "per_op": {k: round(v / max(1, C["ops"]), 3) for k, v in C.items()},
           "per_reach_levels": round(C["reach_levels"] / max(1, C["reach_calls"]), 2),
           "size_hist_16": dict(sorted(sizes.items()))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
