#!/bin/bash
# GPU box: prove_seam per call with the h producer's stage stamps (which regime, 64 or 70 ms, and where H lands)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/r4seamstamps && mkdir -p $O || exit 9
for i in 1 2; do
  BH_HOST_TIMING=1 timeout -k 10 240 python3 -u tools/seam_benchctx.py keep > $O/run_$i.log 2>&1 || { echo "$i failed"; exit 1; }
done
grep -h "call\|keep" $O/run_*.log
