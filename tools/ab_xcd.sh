#!/bin/bash
# XCD-aware WG-stripe map on/off for the default kernel (run via gpurun).
set -euo pipefail
for X in 0 1 0 1; do
  NW_XCD=$X timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/abx.log 2>&1
  python3 -c "import json; j=json.loads(open('gpurun_out/abx.log').read().strip().splitlines()[-1]); print('NW_XCD=$X', j['roofline']['kernel_ms'], 'ms', j['value'], 'GCUPS')"
done
