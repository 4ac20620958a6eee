#!/bin/bash
# Round 5, after the boundary sweeps (k_bsweep, on by default on S1s only):
# the S1s line with its CPU baseline, and the drop-in's first call.
set -o pipefail
D=gpurun_out/r05final6
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 python3 -u bench.py --config S1s > $D/bench_S1s.json 2> $D/bench_S1s.err || exit 91
timeout -k 10 200 python3 -u tools/s3_end_to_end.py S1s > $D/s3e2e.json 2> $D/s3e2e.err || exit 92
timeout -k 10 200 python3 -u bench.py --config S1 --no-cpu-baseline > $D/bench_S1.json 2> $D/bench_S1.err || exit 93
