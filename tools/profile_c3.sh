#!/bin/bash
# profile_c3.sh TAG [bench args...] -- rocprofv3 kernel stats + separate
# FETCH_SIZE / WRITE_SIZE PMC passes of bench.py (default config C3), written
# under gpurun_out/prof_TAG/ (MI355X_MICROARCH.md: counters in their own
# passes, kernel trace/stats only otherwise).
set -o pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $out/bench_under_rocprof.json 2> $out/stats.err || exit 99
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-batches 0 --parity-samples 0 "$@" > $out/fetch.out 2> $out/fetch.err || exit 99
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-batches 0 --parity-samples 0 "$@" > $out/write.out 2> $out/write.err || exit 99
find $out -name "*.csv" | head -20
