#!/bin/bash
# round-4 call 21: the default batch 1024 -- GPU suite, the default line (CPU
# baseline, parity, host-to-host), the C3 profile at B = 1024 (kernel trace +
# stats, FETCH / WRITE passes), C4's strong-scaling job on one GPU
export TMPDIR=/tmp
o=gpurun_out/r04c21
mkdir -p $o
S=tools/gpu_step.sh
$S 900 $o/gputests.log python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
$S 600 $o/C3_default.json python3 bench.py || exit 99
bash tools/profile_c3.sh r04b || exit 99
$S 400 $o/C4_strong.json python3 bench.py --fixed-timesteps 5000 --steps 2 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
