#!/bin/bash
# GPU box: G1-LDS variant GPU suite + A/B, then the seam traces
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && bash tools/r4_g1ab.sh && bash tools/r4_seam.sh
