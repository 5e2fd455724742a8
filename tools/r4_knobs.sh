#!/bin/bash
# GPU box: resident 2^22 A/B of scheduling knobs at the round-4 defaults (3 alternating runs each)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/r4knobs && mkdir -p $O &&
rm -rf gpurun_out/ab && AB_VARIANTS="def: tail0: tail128: sidelo: g2fill:" AB_ENV_tail0="BH_TAIL_CUS=0" AB_ENV_tail128="BH_TAIL_CUS=128" AB_ENV_sidelo="BH_SIDE_PRIORITY=0" AB_ENV_g2fill="BH_ACC_FILL_G2=0.75" AB_REPS=3 timeout -k 10 900 bash tools/ab_lib.sh > $O/ab.log 2>&1
cp -r gpurun_out/ab $O/ 2>/dev/null; true
