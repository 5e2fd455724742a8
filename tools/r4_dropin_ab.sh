#!/bin/bash
# GPU box: drop-in (bh_prove from host buffers) H placement A/B: default (mode 5 from host buffers)
# against BH_H_MODE=2 (round 3's), alternating, 3 runs each; bench legs: resident + drop-in
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/r4dab && mkdir -p $O || exit 9
for i in 1 2 3; do
  for v in def m2; do
    if [ $v = m2 ]; then E="BH_H_MODE=2"; else E="BH_NOP=1"; fi
    env $E timeout -k 10 300 python3 bench.py --cpu-baseline 0 --c5 0 --seam 0 --steps 10 --warmup 2 > $O/${v}_$i.log 2>&1 || { echo "$v $i failed"; exit 1; }
    python3 - "$v" "$O/${v}_$i.log" >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1], d["ms_per_step"], d["dropin"]["ms_per_step"], round(d["dropin"]["ms_per_step"] / d["ms_per_step"], 4))
PY
  done
done
