#!/bin/bash
# round-4 call 35: the smoothed-prolongator transfers (k_restrict0_sa,
# k_prolong0_sa) with more systems per workgroup / thread -- V bit-identity
# (S1s, 97 timesteps, batches 97 and 40) and per-kernel times on S1
export TMPDIR=/tmp
o=gpurun_out/r04c35
mkdir -p $o
S=tools/gpu_step.sh
for v in base v1 v2 v3; do
  if [ $v = base ]; then L=""; else L="MOFHIP_LIB=abvar/libmofhip_$v.so"; fi
  env $L timeout -k 10 120 python3 tools/vhash.py S1s 98 > $o/vhash_$v.json 2> $o/vhash_$v.err || exit 99
  env $L timeout -k 10 120 python3 tools/vhash.py S1s 98 40 > $o/vhash40_$v.json 2> $o/vhash40_$v.err || exit 99
done
prof() {  # tag env...
  local tag=$1; shift
  mkdir -p $o/$tag
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$tag -o run -- \
      python3 bench.py --config S1 --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/$tag/bench.json 2> $o/$tag/err.txt || exit 99
}
prof base MOF_DUMMY=0
prof v1 MOFHIP_LIB=abvar/libmofhip_v1.so
prof v2 MOFHIP_LIB=abvar/libmofhip_v2.so
prof v3 MOFHIP_LIB=abvar/libmofhip_v3.so
