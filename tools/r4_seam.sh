#!/bin/bash
# GPU box: kernel traces of one resident / drop-in / seam proof each (tools/seam_trace.py), seam probe
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4seam} && mkdir -p $O &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/seam_trace.py 22 > $O/trace.log 2>&1 &&
timeout -k 10 300 python3 tools/seam_probe.py 22 4 > $O/probe.log 2>&1
