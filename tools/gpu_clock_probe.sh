#!/bin/bash
# GPU box: engine clock and power while the 2^22 bench runs (rocm-smi sampled every ~0.2 s, read only),
# plus the list of PMC counters this rocprofv3 offers.  Output: gpurun_out/clock/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/clock
mkdir -p $O
timeout -s KILL 90 rocprofv3 -L > $O/counters.txt 2>&1 || true
rocm-smi --showclocks --showpower > $O/idle.txt 2>&1
( for i in $(seq 1 150); do date +%s.%N; rocm-smi --showclocks --showpower 2>&1 | grep -E "sclk|Power|fclk|mclk"; sleep 0.2; done ) > $O/samples.txt 2>&1 &
SP=$!
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --c5 0 --dropin 0 --steps 200 --warmup 2 > $O/bench.log 2>&1
rc=$?
kill $SP 2>/dev/null
wait $SP 2>/dev/null
exit $rc
