#!/bin/bash
# Round 3, late session (GPU box, repo root): clock under load, PMC passes (incl. GRBM for the
# held clock), and the N = 8 rehearsal with and without BH_LAST_HALVES.  Output: gpurun_out/{clock,pmc,abreh}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/gpu_clock_probe.sh || exit $?
bash tools/gpu_pmc.sh || exit $?
REH_VARIANTS="default halves" REH_ENV_default="BH_LAST_HALVES=0" REH_ENV_halves="BH_LAST_HALVES=1" REH_REPS=2 bash tools/ab_rehearsal.sh
