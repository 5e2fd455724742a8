#!/bin/bash
# A/B of prover scheduling knobs on one box (bench.py, 2^22 proof); results in gpurun_out/ab/
set -e
mkdir -p gpurun_out/ab
run() { name=$1; shift; env "$@" timeout -k 10 120 python bench.py --cpu-baseline 0 --steps 8 --warmup 2 > gpurun_out/ab/$name.log 2>&1; }
for cfg in "$@"; do
  name=${cfg%%:*}; vars=${cfg#*:}
  run "$name" $vars
done
