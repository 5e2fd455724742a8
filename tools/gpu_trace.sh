#!/bin/bash
# GPU box: kernel traces of the 2^22 bench proofs, overlapped (default schedule) and
# serialised (BH_PROVER_SERIAL=1).  Output: gpurun_out/trace/{ovl,serial}/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/trace
mkdir -p $O
set -e
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ovl -o run -- python3 bench.py --cpu-baseline 0 --c5 0 --dropin 0 --steps 3 --warmup 1 > $O/ovl.log 2>&1
[ "${SKIP_SERIAL:-0}" = 1 ] || BH_PROVER_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- python3 bench.py --cpu-baseline 0 --c5 0 --dropin 0 --steps 3 --warmup 1 > $O/serial.log 2>&1
