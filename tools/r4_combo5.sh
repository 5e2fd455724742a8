#!/bin/bash
# GPU box: the direct-G2 subprocess test, then the seam probe with the h producer's stage timing
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/r4c5 && mkdir -p $O &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 280 --timeout-method thread -k "g2_direct" > $O/pytest_g2direct.log 2>&1 &&
BH_HOST_TIMING=1 timeout -k 10 300 python3 tools/seam_probe.py 22 4 > $O/probe.log 2>&1
