#!/bin/bash
# round-4 call 17: the default batch on the final build (C3 at B = 384 / 512 /
# 768 / 1024, one box)
export TMPDIR=/tmp
o=gpurun_out/r04c17
mkdir -p $o
S=tools/gpu_step.sh
for b in 512 768 384 1024 512; do
  $S 300 $o/c3_b${b}_$RANDOM.json python3 bench.py --batch $b --steps 6 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
done
