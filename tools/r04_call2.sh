#!/bin/bash
# round-4 call 2: the configuration lines (CPU baselines timed in full on the
# small jobs, a 64-process pool on C3), the S1-like meshes, R3
o=gpurun_out/r04c2
mkdir -p $o
S=tools/gpu_step.sh
$S 400 $o/bench_C1.json python3 bench.py --config C1 --steps 20 --warmup 2 || exit 99
$S 500 $o/bench_S1s.json python3 bench.py --config S1s --steps 20 --warmup 2 || exit 99
$S 400 $o/bench_S1.json python3 bench.py --config S1 --steps 6 --warmup 2 --no-cpu-baseline || exit 99
$S 400 $o/bench_R3.json python3 bench.py --config R3 --steps 4 --warmup 1 --no-cpu-baseline || exit 99
$S 600 $o/bench_C3_cpu64.json python3 bench.py --steps 10 --warmup 2 --cpu-cores 64 --cpu-timesteps-per-core 1 || exit 99
