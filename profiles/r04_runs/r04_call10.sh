#!/bin/bash
# round-4 call 10: the first refinement step's inner tolerance (bench
# --inner-rtol) on the S1-like patch, C3 and R3: the second inner solve starts
# on a residual without the easy modes, so a deeper first solve may save more
# iterations than it costs
export TMPDIR=/tmp
o=gpurun_out/r04c10
mkdir -p $o
S=tools/gpu_step.sh
for cfg in S1 C3 R3; do
  for it in 1e-4 1e-5 1e-6 1e-7; do
    $S 300 $o/${cfg}_ir$it.json python3 bench.py --config $cfg --steps 3 --warmup 1 --inner-rtol $it --no-cpu-baseline --parity-samples 1 --host-batches 0 || exit 99
  done
done
