#!/bin/bash
# Pair kernel at 100k^2: WG-stripe size (compute waves per workgroup) vs the
# balanced one-WG-per-CU plan.  Fewer, fuller WG-stripes mean fewer granule
# hand-offs along the stripe chain.  Run via gpurun from the repo root:
#   bash tools/ab_pair_waves.sh [W ...]
set -euo pipefail
mkdir -p gpurun_out
export NW_KERNEL=pair
WS=${*:-"0 4 6 8"}
for W in $WS; do
  if [ "$W" = 0 ]; then unset NW_WAVES; else export NW_WAVES=$W; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/abw_$W.log 2>&1
  echo "W=$W: $(python3 -c "import json; j=json.loads(open('gpurun_out/abw_$W.log').read().strip().splitlines()[-1]); print(j['value'], 'GCUPS', j['roofline']['kernel_ms'], 'ms kernel, frac', j['roofline']['frac'], 'waves', j['config']['waves_per_wg'])")"
done
for W in $WS; do
  if [ "$W" = 0 ]; then unset NW_WAVES; else export NW_WAVES=$W; fi
  echo "--- trace W=$W"
  timeout -k 10 120 python tools/trace_fill.py 100000 100000 sd
done
