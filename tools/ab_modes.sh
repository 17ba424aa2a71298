#!/bin/bash
# Full-load kernel time per output mode on one box (100k x 100k): what storing
# scores / codes costs beyond computing them (t = stats only: codes and scores
# computed, nothing stored).
for r in 1 2; do
  for o in sd s d t _; do
    oo=$o; [ "$o" = "_" ] && oo=""
    printf "round %d outputs=%-3s " $r "'$oo'"
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --outputs "$oo" | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["roofline"]["kernel_ms"])'
  done
done
