#!/bin/bash
# GPU box: C5 (64 x 2^20) with 2 vs 3 pipelined lanes at the round-4 defaults (first accumulation on its own stream)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/r4c5lanes && mkdir -p $O || exit 9
for i in 1 2; do
  for L in 2 3; do
    timeout -k 10 300 python3 bench.py --cpu-baseline 0 --dropin 0 --steps 3 --warmup 2 --c5-lanes $L > $O/L${L}_$i.log 2>&1 || { echo "L$L $i failed"; exit 1; }
    python3 - "L$L" "$O/L${L}_$i.log" >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1], d["ms_per_step"], d["c5"]["ms_per_proof"], d["c5"]["proofs_match_single"])
PY
  done
done
cat $O/summary.txt
