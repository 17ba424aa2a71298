#!/bin/bash
# One library, several settings of an environment knob, on a bench workload
# (run via gpurun):  bash tools/ab_env.sh NW_HEAD_PACE "0 2 4 8" [bench.py args...]
set -euo pipefail
VAR=$1; VALS=$2; shift 2
for rep in 1 2; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 200 python bench.py --no-cpu-baseline --no-c2 "$@" > gpurun_out/env.log 2>&1
    python3 -c "import json; j=json.loads(open('gpurun_out/env.log').read().strip().splitlines()[-1]); print('$VAR=$v', j['roofline']['kernel_ms'], 'ms', j['value'], 'GCUPS', j.get('parity', {}).get('ok'))"
  done
done
