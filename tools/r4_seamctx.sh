#!/bin/bash
# GPU box: the bench's seam leg with and without the C5 leg run before it on the same context
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/r4seamctx && mkdir -p $O || exit 9
for i in 1 2; do
  for C in 0 64; do
    timeout -k 10 300 python3 bench.py --cpu-baseline 0 --steps 5 --warmup 2 --c5 $C > $O/c${C}_$i.log 2>&1 || { echo "c5=$C $i failed"; exit 1; }
    python3 - "c5=$C" "$O/c${C}_$i.log" >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1], d["ms_per_step"], d["dropin"]["ms_per_step"], d["dropin"]["seam"]["ms_per_step"], d["dropin"]["seam"]["vs_dropin"])
PY
  done
done
cat $O/summary.txt
