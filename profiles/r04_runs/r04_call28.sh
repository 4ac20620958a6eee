#!/bin/bash
# round-4 call 28: the N-rank launcher rehearsed on one GPU (2 ranks, gloo
# barrier; the HBM guard halves each rank's batch)
export TMPDIR=/tmp
o=gpurun_out/r04c28
mkdir -p $o
S=tools/gpu_step.sh
MOF_BENCH_REHEARSE=1 $S 600 $o/C3_rehearse_n2.json python3 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
