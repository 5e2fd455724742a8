#!/bin/bash
# GPU box: rehearsal A/B of environment variants at N = 8 and N = 2 (ranks 0 and N-1)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4rehab} && mkdir -p $O || exit 9
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u tools/shard_rehearsal.py --shards ${REH_SHARDS:-1,2,8} --reps 3 > $O/$n.log 2>&1 || { echo "$n failed"; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v["max"] for k, v in d["per_rank_ms"].items()}, d.get("predicted_speedup"))')" >> $O/summary.txt
}
run base BH_NOP=1
run dhcu0 BH_DIST_H_CUS=0
run tc20 BH_TABLE_C=20
run lar2 BH_LAST_ACC_ROUNDS=2
run hm4 BH_H_MODE=4
run g2d BH_G2_DIRECT=1
run base2 BH_NOP=1
