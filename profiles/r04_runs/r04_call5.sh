#!/bin/bash
# round-4 call 5: the GPU suite; the configuration lines of this build (CPU
# baselines: C1 / S1s timed in full, C3 on 16 and on 64 pool processes)
o=gpurun_out/r04c5
mkdir -p $o
S=tools/gpu_step.sh
$S 600 $o/gputests.log python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread || exit 99
$S 400 $o/C3_default.json python3 bench.py || exit 99
$S 300 $o/C1.json python3 bench.py --config C1 --steps 20 --warmup 2 || exit 99
$S 500 $o/S1s.json python3 bench.py --config S1s --steps 20 --warmup 2 || exit 99
$S 400 $o/S1.json python3 bench.py --config S1 --steps 4 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 400 $o/R3.json python3 bench.py --config R3 --steps 4 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 300 $o/C2.json python3 bench.py --config C2 --steps 8 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
$S 700 $o/C3_cpu64.json python3 bench.py --steps 8 --warmup 2 --host-batches 0 --cpu-cores 64 --cpu-timesteps-per-core 1 || exit 99
