#!/bin/bash
# GPU box: multi-GPU rehearsal at 2^22 (every rank) and C4 (2^24, ranks 0 and 7), and a kernel
# trace of serialised proofs (BH_PROVER_SERIAL=1: per-kernel costs without overlap).
# Output: gpurun_out/measure/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/measure
mkdir -p $O
set -e
timeout -k 10 400 python -u tools/shard_rehearsal.py --shards 1,2,4,8 --all-ranks 1 > $O/rehearsal_2p22.log 2>&1
BH_PROVER_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- python3 bench.py --cpu-baseline 0 --c5 0 --dropin 0 --steps 3 --warmup 1 > $O/serial_bench.log 2>&1
[ "${SKIP_C4:-0}" = 1 ] || timeout -k 10 500 python -u tools/shard_rehearsal.py --log-constraints 24 --shards 8 --reps 3 > $O/rehearsal_2p24.log 2>&1
