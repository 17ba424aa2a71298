#!/bin/bash
# Every lib_ab/*.so on the bench workload (run via gpurun):
#   bash tools/ab_libs.sh [tools/ab_run.py options, e.g. --outputs sd,none]
exec python3 tools/ab_run.py --libs 'lib_ab/*.so' "$@"
