#!/bin/bash
# GPU box: GPU suite with the direct G2 kernel, A/B of G2-direct and G1-LDS against the in-tree
# default, the N = 1..8 rehearsal, the seam traces
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4c2} && mkdir -p $O &&
BH_G2_DIRECT=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_g2direct.log 2>&1 &&
rm -rf gpurun_out/ab && AB_VARIANTS="cur: dir: g1lds:abl/libbellman_hip_g1lds.so" AB_ENV_dir="BH_G2_DIRECT=1" AB_REPS=3 timeout -k 10 600 bash tools/ab_lib.sh > $O/ab.log 2>&1 &&
cp -r gpurun_out/ab $O/ && TAG=${TAG:-r4c2}/reh bash tools/r4_reh.sh &&
TAG=${TAG:-r4c2}/seam bash tools/r4_seam.sh
cp -r gpurun_out/ab $O/ 2>/dev/null; true
