set -o pipefail
for v in "K3:0" "K2:16" "K2:0"; do
  lib=${v%%:*}; st=${v##*:}
  PAXISIM_STAGE=$st PAXISIM_LIB=$PWD/paxi_amd/variants/lib$lib.so timeout -k 10 100 python bench.py --no-cpu-baseline --steps 4 --warmup 2 > /tmp/o.json 2>/dev/null || { echo fail; exit 1; }
  python3 -c "import json;d=json.load(open('/tmp/o.json'));c=d['config'];print('$v', '%.3g msg/s'%d['value'], '%.2f ms/launch'%d['roofline']['avg_launch_ms'], c['tiles_per_cu'], c['lds_per_tile'], c['staged_msgs'])"
done
