# round 4: full GPU suite + the default bench line (TAG names the output dir)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4i} && mkdir -p $O &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
