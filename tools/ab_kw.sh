#!/bin/bash
# Kernel x waves per workgroup on one bench shape (run via gpurun):
#   bash tools/ab_kw.sh L1 L2 "scan:4 skew:2 skew:4" [bench.py args...]
set -euo pipefail
L1=$1; L2=$2; KWS=$3; shift 3
for kw in $KWS; do
  k=${kw%%:*}; w=${kw##*:}
  NW_KERNEL=$k NW_WAVES=$w timeout -k 10 200 python bench.py --no-cpu-baseline --no-c2 --L1 "$L1" --L2 "$L2" "$@" > gpurun_out/kw.log 2>&1
  python3 -c "import json; j=json.loads(open('gpurun_out/kw.log').read().strip().splitlines()[-1]); print('${L1}x${L2} $k W=$w', j['roofline']['kernel_ms'], 'ms', j['value'], 'GCUPS', j.get('parity', {}).get('ok'))"
done
