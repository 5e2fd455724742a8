#!/bin/bash
# GPU box: the C4 sharded test under several library builds (diagnosis)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${TAG:-r4diag} && mkdir -p $O
T="tests/test_gpu_parity.py::test_c4_2p24_sharded_8_ways_equals_single_device_proof"
VARS=${DIAG_VARIANTS:-"new: inl:abl/libbellman_hip_inl.so base:abl/libbellman_hip_base.so"}
for v in $VARS; do
  n=${v%%:*}; p=${v#*:}
  if [ -n "$p" ]; then export BH_LIB_OVERRIDE=$GRAFT_REPO_ROOT/$p; else unset BH_LIB_OVERRIDE; fi
  timeout -k 10 300 python -u -m pytest $T ${DIAG_EXTRA} -x -q --timeout 250 --timeout-method thread > $O/$n.log 2>&1
  rc=$?; echo "$n rc=$rc $(tail -1 $O/$n.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
