#!/bin/bash
# Round 5 final measurements, part C: the configurations the smoothed-P
# Galerkin / restriction changes touch (S1, R3, S1s, F3), and S1's rocprof
# kernel stats, on the final build.
set -o pipefail
D=gpurun_out/r05final3
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 240 python3 -u bench.py --config S1 --steps 5 --no-cpu-baseline > $D/bench_S1.json 2> $D/bench_S1.err || exit 91
timeout -k 10 240 python3 -u bench.py --config R3 --steps 5 --no-cpu-baseline > $D/bench_R3.json 2> $D/bench_R3.err || exit 92
timeout -k 10 200 python3 -u bench.py --config S1s > $D/bench_S1s.json 2> $D/bench_S1s.err || exit 93
timeout -k 10 400 python3 -u bench.py --config F3 --steps 10 > $D/bench_F3.json 2> $D/bench_F3.err || exit 94
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_S1 -o run -- \
    python3 bench.py --config S1 --steps 3 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
    > $D/prof_S1.json 2> $D/prof_S1.err || exit 95
