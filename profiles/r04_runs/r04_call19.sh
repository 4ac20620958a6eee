#!/bin/bash
# round-4 call 19: the default batch on the final build, interleaved on one box
export TMPDIR=/tmp
o=gpurun_out/r04c19
mkdir -p $o
S=tools/gpu_step.sh
for rep in 1 2; do
  for b in 512 768 1024; do
    $S 300 $o/c3_b${b}_r$rep.json python3 bench.py --batch $b --steps 8 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
  done
done
