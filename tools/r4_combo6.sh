#!/bin/bash
# GPU box: direct-G2 subprocess test, seam probe with producer timing, drop-in H placement A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && bash tools/r4_combo5.sh && bash tools/r4_dropin_ab.sh
