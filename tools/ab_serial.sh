#!/bin/bash
# GPU box: same-box A/B of library builds, per kernel, with the prover serialised on one stream
# (BH_PROVER_SERIAL=1: each kernel's duration without overlap) -- rocprofv3 kernel stats of a
# short 2^22 bench per variant.  AB_VARIANTS as in tools/ab_lib.sh (name:path, empty = in-tree).
# Output: gpurun_out/abs/<name>/ (stats CSV) and gpurun_out/abs/summary.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/abs
mkdir -p $O
VARIANTS=${AB_VARIANTS:-"base:abl/libbellman_hip_base.so new:"}
for vp in $VARIANTS; do
  v=${vp%%:*}
  p=${vp#*:}
  if [ -n "$p" ]; then export BH_LIB_OVERRIDE=$GRAFT_REPO_ROOT/$p; else unset BH_LIB_OVERRIDE; fi
  BH_PROVER_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- \
    python3 bench.py --cpu-baseline 0 --c5 0 --dropin 0 --steps 3 --warmup 1 ${AB_ARGS} > $O/${v}_bench.log 2>&1 || exit $?
  python3 - "$v" $O/$v >> $O/summary.txt <<'PY'
import csv, glob, sys
name, d = sys.argv[1], sys.argv[2]
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(name, r["Name"][:60].replace(" ", ""), r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms avg",
          round(float(r["TotalDurationNs"]) / 1e6, 2), "ms total")
PY
done
