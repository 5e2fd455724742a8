#!/bin/bash
# GPU box: kernel traces of ranks of the N-GPU rehearsal (RANK_SPECS "N:k ...", default 8:4).
# Output: gpurun_out/rank/<N>_<k>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/rank
mkdir -p $O
for spec in ${RANK_SPECS:-8:4}; do
  d=$O/${spec/:/_}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/shard_rehearsal.py --rank-only $spec --reps 3 > $d.log 2>&1 || exit $?
done
