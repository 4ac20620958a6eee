#!/bin/bash
# Round 5 final measurements on the final build (early convergence marking,
# compacted tail launches, slab Galerkin, sorted restriction), part 1: the
# C3 default line, its rocprof stats / trace and FETCH / WRITE PMC passes,
# F3 with its CPU baseline, S1 and R3.
set -o pipefail
D=gpurun_out/r05final4
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > $D/bench_C3_default.json 2> $D/bench_C3_default.err || exit 91
bash tools/profile_c3.sh r05d || exit 92
timeout -k 10 400 python3 -u bench.py --config F3 --steps 10 > $D/bench_F3.json 2> $D/bench_F3.err || exit 93
timeout -k 10 240 python3 -u bench.py --config S1 --steps 5 --no-cpu-baseline > $D/bench_S1.json 2> $D/bench_S1.err || exit 94
timeout -k 10 240 python3 -u bench.py --config R3 --steps 5 --no-cpu-baseline > $D/bench_R3.json 2> $D/bench_R3.err || exit 95
