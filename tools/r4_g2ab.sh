#!/bin/bash
# GPU box: GPU suite on the in-tree build, then same-box A/B of the G2 accumulation variants
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4g2} && mkdir -p $O &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
AB_VARIANTS="${AB_VARIANTS:-base:abl/libbellman_hip_base.so new:}" AB_REPS=${AB_REPS:-3} timeout -k 10 900 bash tools/ab_lib.sh > $O/ab.log 2>&1
cp -r gpurun_out/ab $O/ 2>/dev/null; true
