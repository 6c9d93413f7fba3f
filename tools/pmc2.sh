#!/bin/bash
# rocprofv3 PMC passes for arbitrary counter groups: tools/pmc2.sh <tag> "<grp1>" "<grp2>" ... -- <bench args>
set -o pipefail
TAG=$1; shift
GROUPS_=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do GROUPS_+=("$1"); shift; done
[ "$1" == "--" ] && shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --stats -d "$OUT/p$i" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --no-shard-check "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  python3 - "$OUT/p$i/run_counter_collection.csv" <<'PY'
import csv, sys, collections
rows=list(csv.DictReader(open(sys.argv[1])))
agg=collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if 'sim_steps' not in r['Kernel_Name'] and 'sim_serial' not in r['Kernel_Name']: continue
    agg[int(r['Dispatch_Id'])][r['Counter_Name']]+=float(r['Counter_Value'])
ds=sorted(agg)[-10:]
import os
kt=os.path.join(os.path.dirname(sys.argv[1]),'run_kernel_trace.csv')
dur=''
if os.path.exists(kt):
    d={int(r['Dispatch_Id']):(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6 for r in csv.DictReader(open(kt)) if int(r['Dispatch_Id']) in ds}
    dur=f" kernel_ms={sum(d.values())/max(1,len(d)):.3f}"
print(' '.join(f"{k}={sum(agg[d][k] for d in ds)/len(ds):.4g}" for k in agg[ds[-1]]) + dur, '(mean of the last', len(ds), 'dispatches)')
PY
done
