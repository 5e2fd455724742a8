#!/bin/bash
# GPU box: GPU suite on the G1-LDS variant build, then same-box A/B against the in-tree build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4g1} && mkdir -p $O &&
BH_LIB_OVERRIDE=$GRAFT_REPO_ROOT/abl/libbellman_hip_g1lds.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_g1lds.log 2>&1 &&
rm -rf gpurun_out/ab && AB_VARIANTS="${AB_VARIANTS:-cur: g1lds:abl/libbellman_hip_g1lds.so}" AB_REPS=${AB_REPS:-3} timeout -k 10 900 bash tools/ab_lib.sh > $O/ab.log 2>&1
cp -r gpurun_out/ab $O/ 2>/dev/null; true
