set -e
for s in "10000 10000" "20000 4000" "100000 12500" "100000 25000" "100000 50000" "100000 100000"; do
  set -- $s
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-c2 --L1 $1 --L2 $2 --steps 10 --warmup 2 > gpurun_out/sh.log 2>&1
  python3 -c "import json; j=json.loads(open('gpurun_out/sh.log').read().strip().splitlines()[-1]); print('$1x$2', 'W', j['config'].get('waves_per_wg'), j['roofline']['kernel_ms'], 'ms', j['value'], 'GCUPS', j.get('parity', {}).get('ok'))"
done
