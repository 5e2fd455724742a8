#!/bin/bash
# GPU box: the C5 throughput leg (bench.py --c5) under variants.  C5_VARIANTS: "name:lanes ...",
# C5_ENV_<name>: environment.  Output: gpurun_out/abc5/summary.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abc5
mkdir -p $O
for vp in ${C5_VARIANTS:-"l2:2"}; do
  v=${vp%%:*}; lanes=${vp#*:}
  envvar="C5_ENV_$v"
  env ${!envvar} timeout -k 10 300 python3 bench.py --log-constraints 20 --steps 2 --warmup 1 --cpu-baseline 0 --dropin 0 --c5 ${C5_N:-32} --c5-lanes $lanes > $O/$v.log 2>&1 || { echo "$v failed"; exit 1; }
  echo "$v $(grep '^{' $O/$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["c5"]["ms_per_proof"], d["c5"]["value"])')" >> $O/summary.txt
  tail -1 $O/summary.txt
done
