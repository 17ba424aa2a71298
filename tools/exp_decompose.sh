#!/bin/bash
# decomposition experiments for the fill kernel
set -e
run() { echo "== $*"; timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@" | python3 -c "import json,sys;j=json.load(sys.stdin);r=j['roofline'];print(j['config']['L1'],j['config']['L2'],j['config']['waves_per_wg'],'GCUPS',j['value'],'kern_ms',r['kernel_ms'],'frac',r['frac'])"; }
run --outputs sd
run --outputs ''
run --outputs s
run --outputs d
run --L1 100000 --L2 6400 --outputs sd
run --L1 100000 --L2 6400 --outputs ''
run --L1 100000 --L2 512 --outputs ''
run --L1 100000 --L2 64 --outputs ''
run --L1 2000 --L2 100000 --outputs sd
run --L1 2000 --L2 100000 --outputs ''
run --L1 10000 --L2 10000 --outputs sd
NW_WAVES=1 run --L1 100000 --L2 6400 --outputs ''
NW_WAVES=4 run --L1 100000 --L2 6400 --outputs ''
