#!/bin/bash
# GPU box helper (round 3): run the steps named in $STEPS (space separated) in order, each under
# its own time limit, into gpurun_out/$TAG/.  A step that times out, aborts or faults ends the
# script (no further GPU step); a test failure (pytest exit 1) does not stop later steps.
#   kfd      KFD topology properties (queue counts) -- no GPU work
#   pytest   the -m gpu suite ($PYTEST_ARGS appended)
#   bench    python bench.py $BENCH_ARGS
#   port22   oracle port at 2^22 -> port_proofs.json fixture (also copied to tests/golden/) + baseline
#   port24   the same at 2^24, added to tests/golden/port_proofs.json
#   rehearse N-rank rehearsal at 2^22 ($REH_ARGS)
#   trace    rocprofv3 kernel trace + stats of a short bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/${TAG:-call}
mkdir -p "$O"
ok() {  # continue only after a clean exit or an ordinary test failure
  local rc=$1
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "step exited $rc: stopping" >> "$O/steps.log"; exit "$rc"; fi
}
for st in ${STEPS:-pytest bench}; do
  echo "$(date +%T) $st" >> "$O/steps.log"
  case $st in
    kfd) (grep -H . /sys/class/kfd/kfd/topology/nodes/*/properties > "$O/kfd_props.txt" 2>&1; true) ;;
    pytest) timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $PYTEST_ARGS > "$O/pytest.log" 2>&1; ok $? ;;
    bench) timeout -k 10 600 python -u bench.py $BENCH_ARGS > "$O/bench.log" 2>&1; ok $? ;;
    port22) timeout -k 10 1100 python -u tools/cpu_baseline_full.py --fixture "$O/port_proofs.json" > "$O/port22.log" 2>&1; ok $?
            cp "$O/port_proofs.json" tests/golden/port_proofs.json ;;
    port24) timeout -k 10 1100 python -u tools/cpu_baseline_full.py --log-constraints 24 --fixture tests/golden/port_proofs.json > "$O/port24.log" 2>&1; ok $?
            cp tests/golden/port_proofs.json "$O/port_proofs.json" ;;
    rehearse) timeout -k 10 600 python -u tools/shard_rehearsal.py $REH_ARGS > "$O/rehearsal.log" 2>&1; ok $? ;;
    trace) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 bench.py --cpu-baseline 0 --c5 0 --dropin 0 --steps 5 --warmup 2 $TRACE_ARGS > "$O/trace_bench.log" 2>&1; ok $? ;;
    *) echo "unknown step $st" >> "$O/steps.log" ;;
  esac
done
echo "$(date +%T) done" >> "$O/steps.log"
