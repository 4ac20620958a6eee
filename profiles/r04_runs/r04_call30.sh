#!/bin/bash
# round-4 call 30: the row assembly with the next incidence's entry loaded
# ahead (bit-identical arithmetic) vs the committed build: per-kernel times
# under rocprof, interleaved; the parity tests on the new build
export TMPDIR=/tmp
o=gpurun_out/r04c30
mkdir -p $o
S=tools/gpu_step.sh
$S 400 $o/parity.log python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread || exit 99
prof() {  # tag env...
  local tag=$1; shift
  mkdir -p $o/$tag
  env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$tag -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/$tag/bench.json 2> $o/$tag/err.txt || exit 99
}
prof base1 MOFHIP_LIB=abvar/libmofhip_base.so
prof new1 MOF_DUMMY=0
prof base2 MOFHIP_LIB=abvar/libmofhip_base.so
prof new2 MOF_DUMMY=0
