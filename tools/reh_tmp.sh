cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/reh7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not c4_2p24" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $O/bench.log 2>&1 || exit 1
for l in 1 3; do timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-baseline 0 --dropin 0 --c5-lanes $l > $O/bench_l$l.log 2>&1 || exit 1; done
