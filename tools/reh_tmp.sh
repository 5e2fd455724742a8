cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/reh5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not c4_2p24" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $O/bench.log 2>&1 || exit 1
for v in "X=0" "BH_LAST_TAIL_THREADS=0" "BH_H_MODE=1"; do
  echo "== $v" >> $O/ab.log
  env $v timeout -k 10 120 python -u tools/shard_rehearsal.py --shards 1,4,8 --reps 7 2>&1 | tail -1 >> $O/ab.log || exit 1
done
