#!/bin/bash
# GPU box: one-GPU rehearsal of the N-GPU run at 2^22 (N = 1, 2, 4, 8, every rank timed)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4reh} && mkdir -p $O &&
timeout -k 10 700 python -u tools/shard_rehearsal.py --shards ${REH_SHARDS:-1,2,4,8} --all-ranks 1 --reps ${REH_REPS:-3} > $O/shard_rehearsal.log 2>&1
