set -o pipefail
for C in 16384 32768 65536; do
  timeout -k 10 100 python bench.py --no-cpu-baseline --config 3 --clusters $C --steps 4 --warmup 1 > /tmp/o.json 2>/dev/null || { echo fail; exit 1; }
  python3 -c "import json;d=json.load(open('/tmp/o.json'));print('ABD C=$C', '%.2f ms/launch'%d['roofline']['avg_launch_ms'])"
done
