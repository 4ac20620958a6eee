# rocprofv3 kernel stats of F3 (folded: both levels smoothed) and S1 at the bench's batch
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/prof_r06_f3; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/f3 -o run -- \
    python3 bench.py --config F3 --steps 3 --warmup 1 --no-cpu-baseline --legs none --host-batches 0 --parity-samples 0 > $o/f3_line.json 2> $o/f3.err || exit 99
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/s1 -o run -- \
    python3 bench.py --config S1 --steps 2 --warmup 1 --no-cpu-baseline --legs none --host-batches 0 --parity-samples 0 > $o/s1_line.json 2> $o/s1.err || exit 99
