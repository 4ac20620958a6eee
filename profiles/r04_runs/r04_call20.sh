#!/bin/bash
# round-4 call 20: B = 1024 / 1536 against 512 (lines with parity), kernel
# stats of 512 and 1024 (where the batch's time goes)
export TMPDIR=/tmp
o=gpurun_out/r04c20
mkdir -p $o
S=tools/gpu_step.sh
for b in 1024 512 1536 1024; do
  $S 400 $o/c3_b${b}_$RANDOM.json python3 bench.py --batch $b --steps 6 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
done
for b in 512 1024; do
  mkdir -p $o/p_b$b
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/p_b$b -o run -- \
      python3 bench.py --batch $b --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/p_b$b/bench.json 2> $o/p_b$b/err.txt || exit 99
done
