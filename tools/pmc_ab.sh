#!/bin/bash
# pmc FETCH pass per variant
export TMPDIR=/tmp
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=$PWD/manifold-based-optical-flow-method_amd/mofhip/libmofhip_$v.so
  out=gpurun_out/pmcab/$v; mkdir -p $out
  MOFHIP_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/b.json 2> $out/err.txt || exit 99
done
