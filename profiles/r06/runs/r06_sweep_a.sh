#!/bin/bash
# r06_sweep_a.sh -- the final build's configuration lines, part A (one GPU)
o=gpurun_out/r06_sweep
mkdir -p $o
S=tools/gpu_step.sh
$S 300 $o/C1.json python3 bench.py --config C1 --steps 20 --warmup 2 --legs none || exit 99
$S 300 $o/S1s.json python3 bench.py --config S1s --steps 20 --warmup 2 --legs none || exit 99
$S 300 $o/C2_f64.json python3 bench.py --config C2 --steps 10 --warmup 2 --no-cpu-baseline --legs none || exit 99
$S 300 $o/C2_mixed.json python3 bench.py --config C2 --precision mixed --steps 10 --warmup 2 --no-cpu-baseline --legs none || exit 99
$S 300 $o/P3.json python3 bench.py --config P3 --steps 8 --warmup 2 --no-cpu-baseline --legs none || exit 99
$S 400 $o/S1.json python3 bench.py --config S1 --steps 6 --warmup 1 --no-cpu-baseline --legs none || exit 99
$S 400 $o/R3.json python3 bench.py --config R3 --steps 6 --warmup 1 --no-cpu-baseline --legs none || exit 99
$S 300 $o/S1m.json python3 bench.py --config S1m --steps 6 --warmup 1 --no-cpu-baseline --legs none || exit 99
