#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/r4seamctx2 && mkdir -p $O || exit 9
for m in keep drop keep drop; do
  timeout -k 10 240 python3 -u tools/seam_benchctx.py $m >> $O/summary.txt 2>&1 || { echo "$m failed"; exit 1; }
done
timeout -k 10 240 python3 -u tools/seam_gc.py >> $O/summary.txt 2>&1 || exit 1
cat $O/summary.txt
