#!/bin/bash
# Round 5 final measurements, part A (C3 default line, its rocprof trace /
# stats and the FETCH / WRITE PMC passes, F3 with its CPU baseline).
set -o pipefail
D=gpurun_out/r05final2
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > $D/bench_C3_default.json 2> $D/bench_C3_default.err || exit 91
bash tools/profile_c3.sh r05b || exit 92
timeout -k 10 400 python3 -u bench.py --config F3 --steps 10 > $D/bench_F3.json 2> $D/bench_F3.err || exit 93
