# round 4: NTT parity (limb-wise butterflies) + golden proofs, a quick bench, the profile passes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4j} && mkdir -p $O &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "fft or domain or compute_h or golden or distributed_h or polynomial or host_buffers" > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --c5 0 --steps 10 --warmup 3 > $O/bench.log 2>&1 &&
TAG=${TAG:-r4j}/prof PSTEPS=2 bash tools/r4_prof.sh
