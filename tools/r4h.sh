# round 4: scratch report test, seam vs bh_prove device timelines
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4h} && mkdir -p $O &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_affine.py -x -v -s --timeout 200 --timeout-method thread -k scratch > $O/tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/seam_trace.py 22 > $O/seam_trace.log 2>&1 &&
python3 tools/split_bursts.py $O/trace/run_kernel_trace.csv 3 50 --min-us 20 > $O/bursts.txt
