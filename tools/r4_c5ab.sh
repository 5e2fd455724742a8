#!/bin/bash
# GPU box: C5 (64 x 2^20, pipelined lanes) with the first accumulation on its own stream vs the main one
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/r4c5ab && mkdir -p $O || exit 9
for i in 1 2; do
  for v in fa main; do
    if [ $v = main ]; then E="BH_FIRST_ACC_STREAM=0"; else E="BH_NOP=1"; fi
    env $E timeout -k 10 300 python3 bench.py --cpu-baseline 0 --dropin 0 --steps 5 --warmup 2 > $O/${v}_$i.log 2>&1 || { echo "$v $i failed"; exit 1; }
    python3 - "$v" "$O/${v}_$i.log" >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1], d["ms_per_step"], d["c5"]["ms_per_proof"])
PY
  done
done
