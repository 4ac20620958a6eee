#!/bin/bash
# round-4 call 34: per-kernel times of the S1-like patch and R3 (where the
# irregular class spends its time)
export TMPDIR=/tmp
o=gpurun_out/r04c34
mkdir -p $o
prof() {  # tag config
  local tag=$1 cfg=$2
  mkdir -p $o/$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$tag -o run -- \
      python3 bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/$tag/bench.json 2> $o/$tag/err.txt || exit 99
}
prof S1 S1
prof R3 R3
