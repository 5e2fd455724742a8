#!/bin/bash
# The round's committed measurements (run on the GPU box from the repo root):
#   GPU tests, the default bench line (with the CPU baseline, C5 and drop-in legs), a kernel trace
#   + stats of the same bench, the multi-GPU rehearsal (every rank, N = 1, 2, 4, 8) and the C4
#   (2^24) rehearsal at N = 8.  PMC passes: tools/gpu_pmc.sh.  Output: gpurun_out/round/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/round
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --cpu-baseline 0 --c5 0 --dropin 0 > $O/bench_trace.log 2>&1
timeout -k 10 400 python -u tools/shard_rehearsal.py --shards 1,2,4,8 --all-ranks 1 > $O/shard_rehearsal.log 2>&1
timeout -k 10 500 python -u tools/shard_rehearsal.py --log-constraints 24 --shards 8 --reps 3 > $O/shard_rehearsal_2p24.log 2>&1
