#!/bin/bash
# GPU box: same-box A/B of library builds on the 2^22 bench (alternating runs).
#   AB_VARIANTS: space-separated name:path pairs (path empty = the in-tree build), default
#   "base:ab/libbellman_hip_base.so new:".  AB_ENV_<name>: extra environment for a variant.
# Output: gpurun_out/ab/<name>_<i>.log and one summary line per run in gpurun_out/ab/summary.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab
mkdir -p $O
VARIANTS=${AB_VARIANTS:-"base:ab/libbellman_hip_base.so new:"}
REPS=${AB_REPS:-3}
ARGS="--cpu-baseline 0 --c5 0 --dropin 0 --steps ${AB_STEPS:-10} --warmup 2 ${AB_ARGS}"
for i in $(seq 1 $REPS); do
  for vp in $VARIANTS; do
    v=${vp%%:*}
    p=${vp#*:}
    envvar="AB_ENV_$v"
    if [ -n "$p" ]; then lib="BH_LIB_OVERRIDE=$GRAFT_REPO_ROOT/$p"; else lib=""; fi
    env $lib ${!envvar} timeout -k 10 300 python3 bench.py $ARGS > $O/${v}_$i.log 2>&1 || { echo "$v $i failed"; exit 1; }
    python3 - "$v" "$O/${v}_$i.log" >> $O/summary.txt <<'EOF'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        dr = d.get("dropin") or {}
        print(sys.argv[1], d["ms_per_step"], "dropin", dr.get("ms_per_step"),
              "landed", (dr.get("landed_ms") or {}).get("per_call", [None])[-1], json.dumps(d["breakdown_ms"]))
EOF
    tail -1 $O/summary.txt
  done
done
