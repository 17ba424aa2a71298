#!/bin/bash
# One GPU-box session: the steps named on the command line, each under its own
# time limit, stopping at the first failure.  Run via gpurun from the repo root:
#   gpurun --timeout 1200 -- bash tools/gpu_session.sh TAG step [step ...]
# steps: newtests | noalloc | tests | bench | ab:<bench args> | shapes
set -uo pipefail
TAG=$1; shift
OUT=gpurun_out
mkdir -p $OUT
run() {  # run LIMIT NAME cmd...
  local lim=$1 name=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/${TAG}_session.txt >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/${TAG}_session.txt >&2
  return $rc
}
PYT="python -u -m pytest -x -v --timeout 180 --timeout-method thread"
for step in "$@"; do
  case "$step" in
    newtests) run 900 newtests $PYT tests/test_gpu_raw.py 2>&1 | tee $OUT/${TAG}_tests_raw.txt || exit 1 ;;
    noalloc)  run 600 noalloc $PYT tests/wip_no_alloc.py 2>&1 | tee $OUT/${TAG}_tests_noalloc.txt || exit 1 ;;
    tests)    run 1100 tests $PYT tests -m gpu 2>&1 | tee $OUT/${TAG}_gpu_tests.txt || exit 1 ;;
    bench)    run 600 bench python bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || { cat $OUT/${TAG}_bench.err; exit 1; }
              cat $OUT/${TAG}_bench.json ;;
    ab:*)     ARGS=${step#ab:}
              for rep in 1 2; do for L in lib_ab/*.so; do
                NW_LIB=$L run 200 "ab $L $ARGS" python bench.py --no-cpu-baseline --no-hash --no-c2 --steps 10 --warmup 2 $ARGS > $OUT/abl.json 2> $OUT/abl.err || { cat $OUT/abl.err; exit 1; }
                python3 -c "import json; j=json.loads(open('$OUT/abl.json').read().strip().splitlines()[-1]); print('$L', '$ARGS', j['roofline']['kernel_ms'], 'ms', j['value'], 'GCUPS')" | tee -a $OUT/${TAG}_ab.txt
              done; done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
