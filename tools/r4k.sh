# round 4: seam phase probe (host timings, back-to-back vs spaced prove_seam), the 2^22 shard
# rehearsal (ranks 0 and N-1) and kernel traces of rank 0 at N = 2 and N = 8
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4k} && mkdir -p $O &&
BH_HOST_TIMING=1 timeout -k 10 300 python3 -u tools/seam_probe.py 22 6 > $O/probe.log 2>&1 &&
timeout -k 10 400 python3 -u tools/shard_rehearsal.py --shards 1,2,4,8 --reps 3 > $O/rehearsal.log 2>&1 &&
for spec in 2:0 8:0; do d=$O/rank_${spec/:/_}; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/shard_rehearsal.py --rank-only $spec --reps 3 > $d.log 2>&1 || exit $?; done
