# round 4: affine-level tests, full-size parity subset, affine bench and its profile (TAG names the output dir)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4c} && mkdir -p $O &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_affine.py -x -v --timeout 200 --timeout-method thread > $O/affine.log 2>&1 &&
BH_AFFINE=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "window_tables_match or prove_batch_equals or c5_batch or degenerate" > $O/parity.log 2>&1 &&
BH_AFFINE=1 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --c5 0 --dropin 0 --seam 0 --steps 10 --warmup 3 > $O/bench_aff.log 2>&1 &&
BH_AFFINE=1 TAG=${TAG:-r4c}/prof PSTEPS=2 bash tools/r4_prof.sh
