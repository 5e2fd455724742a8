#!/bin/bash
# GPU box, round 4's closing measurements: GPU suite, smoke, the default bench line, a kernel
# trace + stats of a short bench.  Output: gpurun_out/r4final3/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/r4final3 && mkdir -p $O &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --cpu-baseline 0 --c5 0 --dropin 0 --steps 5 --warmup 2 > $O/trace.log 2>&1
