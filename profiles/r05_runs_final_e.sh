#!/bin/bash
# Round 5 final measurements, part 2: the other configurations.
set -o pipefail
D=gpurun_out/r05final4
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 python3 -u bench.py --config S1s > $D/bench_S1s.json 2> $D/bench_S1s.err || exit 91
timeout -k 10 200 python3 -u bench.py --config C1 > $D/bench_C1.json 2> $D/bench_C1.err || exit 92
timeout -k 10 200 python3 -u bench.py --config C2 --steps 5 --no-cpu-baseline > $D/bench_C2_f64.json 2> $D/bench_C2_f64.err || exit 93
timeout -k 10 200 python3 -u bench.py --config C2 --precision mixed --steps 5 --no-cpu-baseline > $D/bench_C2_mixed.json 2> $D/bench_C2_mixed.err || exit 94
timeout -k 10 300 python3 -u bench.py --config C5 --steps 3 --no-cpu-baseline --parity-samples 0 > $D/bench_C5.json 2> $D/bench_C5.err || exit 95
timeout -k 10 300 python3 -u bench.py --fixed-timesteps 5000 --steps 1 --warmup 1 --no-cpu-baseline > $D/bench_C4_strong_n1.json 2> $D/bench_C4_strong_n1.err || exit 96
timeout -k 10 240 python3 -u bench.py --config P3 --steps 5 --no-cpu-baseline > $D/bench_P3.json 2> $D/bench_P3.err || exit 97
