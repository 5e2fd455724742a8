#!/bin/bash
# Round 3's committed measurements, part 2 (GPU box): the one-GPU rehearsal of the multi-GPU run
# at 2^22 (N = 1, 2, 4, 8, every rank timed) and C4 (2^24) at N = 8.  Output: gpurun_out/r3reh/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r3reh
mkdir -p $O
timeout -k 10 560 python -u tools/shard_rehearsal.py --shards 1,2,4,8 --all-ranks 1 --reps 3 > $O/shard_rehearsal.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/shard_rehearsal.py --log-constraints 24 --shards 8 --reps 3 --all-ranks 1 > $O/shard_rehearsal_2p24.log 2>&1
