#!/bin/bash
# Profile the bench workload on the GPU box (run via gpurun from the repo root):
#   bash tools/profile_round.sh r02 [L1 L2]
# Three rocprofv3 runs of bench.py -- kernel trace + stats (the bench's own
# default --steps 20 --warmup 5, so the steady-state kernel average can be
# compared with the line it prints), then WRITE_SIZE and
# FETCH_SIZE in passes of their own (never combined with other tracing) -- then
# tools/pmc_traffic.py writes profiles/<round>_kernel_stats.csv and
# profiles/<round>_pmc_traffic.json.  Each GPU step has its own time limit and
# the chain stops at the first failure.
set -euo pipefail
RND=${1:?round tag}
L1=${2:-100000}
L2=${3:-100000}
OUT=gpurun_out/prof_$RND
export TMPDIR=/tmp
rm -rf "$OUT"
mkdir -p "$OUT"
B=(bench.py --L1 "$L1" --L2 "$L2" --no-cpu-baseline --no-c2)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
    python3 "${B[@]}" --steps 20 --warmup 5 > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/wr" -o run -- \
    python3 "${B[@]}" --no-hash --steps 2 --warmup 0 > "$OUT/wr.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/rd" -o run -- \
    python3 "${B[@]}" --no-hash --steps 2 --warmup 0 > "$OUT/rd.log" 2>&1
python3 tools/pmc_traffic.py "$RND" "$OUT" "$L1" "$L2" 5
