#!/bin/bash
# Round-5 GPU call P: what the arena's placement changes.  Config 3 in four placements -
# plain twice in a row (the two run modes), behind a freed 120 GB pad, physically contiguous - each
# with a translation pass (UTCL1 hits/misses, UTCL2 busy) and a DRAM-request pass.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5p
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -1 "$O/$n.log" | cut -c1-400
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
T="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
D="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum"
B="-- --config 3 --warmup 5 --steps 3"
for k in 1 2 3 4; do step plain_t$k 300 bash tools/pmc2.sh r5p_plain_t$k "$T" $B; step plain_d$k 300 bash tools/pmc2.sh r5p_plain_d$k "$D" $B; done
step pad_t 300 env PAXISIM_ARENA_PAD_MB=120000 bash tools/pmc2.sh r5p_pad_t "$T" $B
step pad_d 300 env PAXISIM_ARENA_PAD_MB=120000 bash tools/pmc2.sh r5p_pad_d "$D" $B
step contig_t 300 env PAXISIM_ARENA_CONTIG=1 bash tools/pmc2.sh r5p_contig_t "$T" $B
step contig_d 300 env PAXISIM_ARENA_CONTIG=1 bash tools/pmc2.sh r5p_contig_d "$D" $B
