set -e
for w in 4 5 6 8 10; do
  NW_WAVES=$w timeout -k 10 100 python bench.py --no-cpu-baseline --no-c2 --steps 10 --warmup 2 > gpurun_out/wv.log 2>&1
  python3 -c "import json; j=json.loads(open('gpurun_out/wv.log').read().strip().splitlines()[-1]); print('W=$w', j['roofline']['kernel_ms'], 'ms', j['value'], 'GCUPS', j['parity']['ok'])"
done
