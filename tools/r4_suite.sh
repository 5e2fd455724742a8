#!/bin/bash
# GPU box: the GPU suite and smoke only (validation of the tree as committed)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/r4suite && mkdir -p $O &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --c5 1 --dropin 0 --steps 10 --warmup 3 > $O/bench.log 2>&1
