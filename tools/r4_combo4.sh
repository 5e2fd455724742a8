#!/bin/bash
# GPU box: GPU suite at the new defaults, the N = 1..8 rehearsal, a rank-0-of-8 kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4c4} && mkdir -p $O &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
TAG=${TAG:-r4c4}/reh bash tools/r4_reh.sh &&
RANK_SPECS="8:0" bash tools/gpu_rank_trace.sh && cp -r gpurun_out/rank $O/
