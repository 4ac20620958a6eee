#!/bin/bash
# config_sweep.sh TAG -- bench lines for the other configurations and modes
# (one GPU), each step under its own time limit, under gpurun_out/sweep_TAG/.
tag=$1
o=gpurun_out/sweep_$tag
mkdir -p $o
S=tools/gpu_step.sh
$S 300 $o/C2_f64.json python3 bench.py --config C2 --steps 10 --warmup 2 --no-cpu-baseline || exit 99
$S 300 $o/C2_mixed.json python3 bench.py --config C2 --precision mixed --steps 10 --warmup 2 --no-cpu-baseline || exit 99
$S 300 $o/P3.json python3 bench.py --config P3 --steps 8 --warmup 2 --no-cpu-baseline || exit 99
$S 400 $o/C5.json python3 bench.py --config C5 --batch 128 --steps 6 --warmup 1 --no-cpu-baseline --parity-samples 0 || exit 99
$S 400 $o/C3_host.json python3 bench.py --io host --steps 10 --warmup 2 --no-cpu-baseline || exit 99
$S 400 $o/C4_strong_n1.json python3 bench.py --fixed-timesteps 5000 --steps 2 --warmup 1 --no-cpu-baseline || exit 99
MOF_BENCH_REHEARSE=1 $S 400 $o/C3_rehearse_n2.json python3 bench.py --gpus 2 --steps 6 --warmup 1 --no-cpu-baseline || exit 99
$S 400 $o/dd_c5_p8.json python3 bench_dd.py --parts 8 --config C5 --batch 64 --steps 3 --warmup 1 || exit 99
$S 400 $o/dd_c5_p8_amg.json python3 bench_dd.py --parts 8 --config C5 --batch 64 --steps 3 --warmup 1 --precond amg || exit 99
$S 400 $o/R3.json python3 bench.py --config R3 --steps 6 --warmup 1 --no-cpu-baseline || exit 99
$S 300 $o/C1.json python3 bench.py --config C1 --steps 20 --warmup 2 --no-cpu-baseline || exit 99
$S 600 $o/rows.jsonl python3 bench_rows.py || exit 99
