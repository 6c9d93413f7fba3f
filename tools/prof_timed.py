"""Average duration of the bench's timed step-kernel launches from a rocprofv3
kernel trace (the last <steps> dispatches of sim_steps), to set beside
bench.py's HIP-event average (roofline.avg_launch_ms).  The --stats summary
averages every dispatch, warm-up included, and warm-up launches are faster
(earlier simulation state).
usage: python tools/prof_timed.py <run_kernel_trace.csv> <timed launches | 0> [bench.json]
(0: the timed launch count is read from bench.json's roofline.launches)"""
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "sim_steps" in r["Kernel_Name"] or "sim_serial" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
steps = int(sys.argv[2])
if steps == 0:
    steps = int(json.load(open(sys.argv[3]))["roofline"]["launches"])
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
names = sorted({r["Kernel_Name"] for r in rows[-steps:]})    # pipelined launches mix sim_serial_pipe and sim_serial
out = {"kernel": names[0] if len(names) == 1 else names, "dispatches": len(d), "timed": steps,
       "rocprof_avg_timed_ms": sum(d[-steps:]) / steps, "rocprof_avg_all_ms": sum(d) / len(d)}
if len(sys.argv) > 3:
    b = json.load(open(sys.argv[3]))
    out["bench_hip_event_avg_ms"] = b["roofline"]["avg_launch_ms"]
    out["ratio"] = out["rocprof_avg_timed_ms"] / out["bench_hip_event_avg_ms"]
print(json.dumps(out, indent=1))
