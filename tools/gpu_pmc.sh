#!/bin/bash
# GPU box: PMC passes over the 2^22 bench (2 proofs), one counter group per run
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass; <= 8 SQ, 4 TCC, 2 GRBM counters).
# GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time = the clock the chip held during the kernel ('DVFS give-back').
# Output: gpurun_out/pmc/<pass>/run_counter_collection.csv
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc
mkdir -p $O
B="--cpu-baseline 0 --c5 0 --dropin 0 --steps 2 --warmup 1"
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- python3 bench.py $B > $O/$n.log 2>&1
}
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU && \
run tcc TCC_HIT_sum TCC_MISS_sum && \
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
