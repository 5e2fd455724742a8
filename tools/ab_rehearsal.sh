#!/bin/bash
# GPU box: the N-GPU rehearsal (every rank) under environment variants, alternating.
#   REH_VARIANTS: names; REH_ENV_<name>: its environment; REH_SHARDS (default 8); REH_REPS (default 1)
# Output: gpurun_out/abreh/<name>_<i>.log, summary.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abreh
mkdir -p $O
for i in $(seq 1 ${REH_REPS:-1}); do
  for v in ${REH_VARIANTS:-default}; do
    envvar="REH_ENV_$v"
    env ${!envvar} timeout -k 10 300 python3 tools/shard_rehearsal.py --shards ${REH_SHARDS:-8} --all-ranks 1 --reps 5 > $O/${v}_$i.log 2>&1 || { echo "$v failed"; exit 1; }
    echo "$v $(tail -1 $O/${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({n: v["max"] for n, v in d["per_rank_ms"].items()}, {n: v["ranks"] for n, v in d["per_rank_ms"].items()})')" >> $O/summary.txt
    tail -1 $O/summary.txt
  done
done
