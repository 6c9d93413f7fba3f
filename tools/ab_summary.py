"""Medians per variant of a tools/ab_env.sh REPS run: value, launch ms, scan s."""
import collections
import json
import os
import statistics
import sys

d = sys.argv[1]
by = collections.defaultdict(list)
for f in sorted(os.listdir(d)):
    if f.endswith(".json") and "_r" in f:
        j = json.load(open(os.path.join(d, f)))
        by[f[:f.rindex("_r")]].append((j["value"], j["roofline"]["avg_launch_ms"],
                                        (j.get("linearizability") or {}).get("scan_s", 0.0)))
out = {}
for n, rs in by.items():
    v, ms, sc = zip(*rs)
    out[n] = {"runs": len(rs), "value_median": statistics.median(v), "value_min": min(v), "value_max": max(v),
              "launch_ms_median": statistics.median(ms), "scan_s_median": statistics.median(sc)}
    print(f"{n:12s} n={len(rs)} value med {statistics.median(v):.4e} [{min(v):.4e}, {max(v):.4e}] "
          f"launch ms med {statistics.median(ms):.2f} scan s med {statistics.median(sc):.3f}")
json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
