#!/bin/bash
# r06_sweep_b.sh -- the final build's configuration lines, part B (one GPU)
o=gpurun_out/r06_sweep
mkdir -p $o
S=tools/gpu_step.sh
$S 400 $o/F3.json python3 bench.py --config F3 --steps 10 --warmup 1 --legs none || exit 99
$S 400 $o/C5.json python3 bench.py --config C5 --batch 512 --steps 4 --warmup 1 --no-cpu-baseline --parity-samples 0 --legs none || exit 99
$S 400 $o/C3_host.json python3 bench.py --io host --steps 10 --warmup 2 --no-cpu-baseline || exit 99
$S 400 $o/C4_strong_n1.json python3 bench.py --fixed-timesteps 5000 --steps 2 --warmup 1 --no-cpu-baseline --legs none || exit 99
MOF_BENCH_REHEARSE=1 $S 400 $o/C3_rehearse_n2.json python3 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline || exit 99
$S 400 $o/dd_c5_p8.json python3 bench_dd.py --parts 8 --config C5 --batch 64 --steps 3 --warmup 1 || exit 99
$S 600 $o/rows.jsonl python3 bench_rows.py || exit 99
