# round 4: input-multiexp device branch + scratch report tests, seam phase probe
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4g} && mkdir -p $O &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_inputs.py tests/test_gpu_affine.py -x -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/seam_probe.py 22 4 > $O/seam.log 2>&1
