#!/bin/bash
# round-4 call 29: system-group size A/B at B=1024 (SpMV, smoother, residual
# G = 4 / 8 / 16), C3 default bench, interleaved
export TMPDIR=/tmp
o=gpurun_out/r04c29
mkdir -p $o
S=tools/gpu_step.sh
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --parity-samples 0"
for r in 1 2; do
  $S 300 $o/g8_$r.json $B || exit 99
  MOFHIP_LIB=abvar/libmofhip_g4.so $S 300 $o/g4_$r.json $B || exit 99
  MOFHIP_LIB=abvar/libmofhip_g16.so $S 300 $o/g16_$r.json $B || exit 99
done
