#!/bin/bash
# GPU box: the -m gpu suite, then the default bench line.  Output: gpurun_out/check/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/check
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1 || exit $?
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/bench.log 2>&1
