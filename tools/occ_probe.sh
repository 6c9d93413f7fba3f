set -o pipefail
export PAXISIM_LIB=$PWD/paxi_amd/variants/libA.so
for W in 8 16; do for C in 16384 32768 49152; do
  timeout -k 10 100 python bench.py --no-cpu-baseline --clusters $C --steps 4 --warmup 1 --window $W > /tmp/o.json 2>/dev/null || { echo fail; exit 1; }
  python3 -c "import json;d=json.load(open('/tmp/o.json'));print('W=$W C=$C', '%.2f ms/launch'%d['roofline']['avg_launch_ms'], d['unfaithful_clusters'])"
done; done
