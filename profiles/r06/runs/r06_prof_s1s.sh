# rocprofv3 kernel trace of S1s (the reference's workload size): where a 97-timestep job's 3.6 ms go
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/prof_r06_s1s; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/s1s -o run -- \
    python3 bench.py --config S1s --steps 20 --warmup 2 --no-cpu-baseline --legs none --host-batches 0 --parity-samples 0 > $o/s1s_line.json 2> $o/s1s.err || exit 99
