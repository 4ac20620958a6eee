#!/bin/bash
# ab_prof.sh TAG VARIANT... -- rocprofv3 kernel stats of a short bench.py
# run for the default build and each mofhip/libmofhip_VARIANT.so, under
# gpurun_out/abprof_TAG/<variant>/ (compare per-kernel averages).
tag=$1; shift
export TMPDIR=/tmp
for v in base "$@"; do
  lib=""
  [ "$v" != base ] && lib=$PWD/manifold-based-optical-flow-method_amd/mofhip/libmofhip_$v.so
  out=gpurun_out/abprof_$tag/$v
  mkdir -p $out
  MOFHIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
      python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 $AB_ARGS > $out/bench.json 2> $out/err.txt || exit 99
done
