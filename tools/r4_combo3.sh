#!/bin/bash
# GPU box: job/seam tests, seam probe, H-placement x G2-kernel A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4c3} && mkdir -p $O &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "seam or async or submit or shared_sorts or deferred or scalars" > $O/pytest_jobs.log 2>&1 &&
timeout -k 10 300 python3 tools/seam_probe.py 22 4 > $O/probe.log 2>&1 &&
rm -rf gpurun_out/ab && AB_VARIANTS="cur: h1: h3: dir: dirh1:" AB_ENV_h1="BH_H_MODE=1" AB_ENV_h3="BH_H_MODE=3" AB_ENV_dir="BH_G2_DIRECT=1" AB_ENV_dirh1="BH_G2_DIRECT=1 BH_H_MODE=1" AB_REPS=3 timeout -k 10 900 bash tools/ab_lib.sh > $O/ab.log 2>&1
cp -r gpurun_out/ab $O/ 2>/dev/null; true
