#!/bin/bash
# Round 3's committed measurements, part 1 (GPU box, repo root): the GPU tests, the default bench
# line (CPU baseline at 2^22, C5, drop-in and seam legs) and a kernel trace + stats of the bench.
# Part 2 (tools/round3_rehearsal.sh): the multi-GPU rehearsals.  Output: gpurun_out/r3/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --cpu-baseline 0 --c5 0 --dropin 0 > $O/bench_trace.log 2>&1
