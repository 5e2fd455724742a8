#!/bin/bash
# GPU box: job/seam tests, seam probe with producer timing, bench drop-in + seam legs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/r4c7 && mkdir -p $O &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "seam or async or submit or shared_sorts or deferred or scalars or host_buffers" > $O/pytest_jobs.log 2>&1 &&
BH_HOST_TIMING=1 timeout -k 10 300 python3 tools/seam_probe.py 22 4 > $O/probe.log 2>&1 &&
timeout -k 10 400 python3 bench.py --cpu-baseline 0 --c5 0 --steps 10 --warmup 2 > $O/bench.log 2>&1
