#!/bin/bash
# r06_sweep_final.sh -- the final build's configuration lines (one GPU)
o=gpurun_out/r06_sweepf
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
$S 400 $o/F3.json python3 bench.py --config F3 --steps 10 --warmup 1 --legs none || exit 99
$S 400 $o/C5.json python3 bench.py --config C5 --batch 512 --steps 4 --warmup 1 --no-cpu-baseline --parity-samples 0 --legs none || exit 99
$S 400 $o/C3_host.json python3 bench.py --io host --steps 10 --warmup 2 --no-cpu-baseline || exit 99
$S 400 $o/C4_strong_n1.json python3 bench.py --fixed-timesteps 5000 --steps 2 --warmup 1 --no-cpu-baseline --legs none || exit 99
MOF_BENCH_REHEARSE=1 $S 400 $o/C3_rehearse_n2.json python3 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline || exit 99
$S 400 $o/dd_c5_p8.json python3 bench_dd.py --parts 8 --config C5 --batch 64 --steps 3 --warmup 1 || exit 99
