#!/bin/bash
# GPU box: the first (G2) accumulation on its own stream (BH_FIRST_ACC_STREAM=1): proof parity subset,
# then A/B against the default
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/r4fa && mkdir -p $O &&
BH_FIRST_ACC_STREAM=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "proofs_golden or c3_family or window_tables_match or prove_batch or host_buffers" > $O/pytest.log 2>&1 &&
rm -rf gpurun_out/ab && AB_VARIANTS="def: fa: fah2:" AB_ENV_fa="BH_FIRST_ACC_STREAM=1" AB_ENV_fah2="BH_FIRST_ACC_STREAM=1 BH_H_MODE=2" AB_REPS=3 timeout -k 10 700 bash tools/ab_lib.sh > $O/ab.log 2>&1
cp -r gpurun_out/ab $O/ 2>/dev/null; true
