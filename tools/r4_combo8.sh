#!/bin/bash
# GPU box: seam with the cyclic GC on/off, then the scheduling-knob A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r4c8 &&
BH_HOST_TIMING=1 timeout -k 10 300 python3 tools/seam_gc.py > gpurun_out/r4c8/seam_gc.log 2>&1 &&
bash tools/r4_knobs.sh
