#!/bin/bash
# The round's committed measurements (run on the GPU box from the repo root):
#   bench line (with the CPU baseline), kernel trace + stats of the same bench, the HBM traffic
#   of the dominant kernel from two separate PMC passes (MI355X_MICROARCH.md: FETCH_SIZE and
#   WRITE_SIZE cannot share a pass), and the one-GPU shard rehearsal.  Output: gpurun_out/round/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/round
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --cpu-baseline 0 > $O/bench_trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --cpu-baseline 0 --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --cpu-baseline 0 --steps 2 --warmup 1 > $O/pmc_write.log 2>&1
timeout -k 10 300 python tools/shard_rehearsal.py --shards 1,2,4,8 --local 1 > $O/shard_rehearsal.log 2>&1
