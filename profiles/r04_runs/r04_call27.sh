#!/bin/bash
# round-4 call 27: the bench with its HBM guard (the default batch must stay
# 1024 on a free MI355X), a short default line
export TMPDIR=/tmp
o=gpurun_out/r04c27
mkdir -p $o
S=tools/gpu_step.sh
$S 400 $o/C3_short.json python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 300 $o/C1.json python3 bench.py --config C1 --steps 5 --warmup 1 --no-cpu-baseline || exit 99
