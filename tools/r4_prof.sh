#!/bin/bash
# GPU box: kernel trace + PMC passes (SQ, FETCH_SIZE, GRBM) of a short 2^22 bench into gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-prof} && mkdir -p $O
B="--cpu-baseline 0 --c5 0 --dropin 0 --seam 0 --steps ${PSTEPS:-2} --warmup 1 $BARGS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $B > $O/trace.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv -d $O/sq -o run -- python3 bench.py $B > $O/sq.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py $B > $O/fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/grbm -o run -- python3 bench.py $B > $O/grbm.log 2>&1
[ -n "$SQW" ] && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR --output-format csv -d $O/sqw -o run -- python3 bench.py $B > $O/sqw.log 2>&1
true
