#!/bin/bash
# One GPU-box session: the steps named on the command line, each under its own
# time limit, stopping at the first failure.  Run via gpurun from the repo root:
#   gpurun --timeout 1200 -- bash tools/gpu_session.sh TAG step [step ...]
# steps: tests | bench | newtests | ab:<tools/ab_run.py options> | run:<command>
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
    newtests) run 900 newtests $PYT ${NEWTESTS:-tests/test_gpu_raw.py} 2>&1 | tee $OUT/${TAG}_tests_new.txt || exit 1 ;;
    tests)    run 1100 tests $PYT tests -m gpu 2>&1 | tee $OUT/${TAG}_gpu_tests.txt || exit 1 ;;
    bench)    run 600 bench python bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || { cat $OUT/${TAG}_bench.err; exit 1; }
              cat $OUT/${TAG}_bench.json ;;
    ab:*)     ARGS=${step#ab:}
              LIBS=(); compgen -G 'lib_ab/*.so' > /dev/null && LIBS=(--libs 'lib_ab/*.so')   # (none built: the in-tree library)
              run 1100 "ab $ARGS" python3 tools/ab_run.py "${LIBS[@]}" $ARGS 2>&1 | tee -a $OUT/${TAG}_ab.txt || exit 1 ;;
    run:*)    CMD=${step#run:}
              run 1100 "$CMD" bash -c "$CMD" 2>&1 | tee -a $OUT/${TAG}_run.txt || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
