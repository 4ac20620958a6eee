#!/bin/bash
# round-4 call 43: the tentative restriction with two members per thread and
# pass (loads in flight together) against the committed build: V hashes (C2
# mesh, S1s), per-kernel times on C3, interleaved
export TMPDIR=/tmp
o=gpurun_out/r04c43
mkdir -p $o
for v in cur base; do
  if [ $v = cur ]; then L=""; else L="MOFHIP_LIB=abvar/libmofhip_$v.so"; fi
  env $L timeout -k 10 120 python3 tools/vhash.py C2 41 > $o/vhash_C2_$v.json 2> $o/vhash_$v.err || exit 99
  env $L timeout -k 10 120 python3 tools/vhash.py S1s 98 40 > $o/vhash_S1s40_$v.json 2>> $o/vhash_$v.err || exit 99
done
prof() {  # tag env...
  local tag=$1; shift
  mkdir -p $o/$tag
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$tag -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/$tag/bench.json 2> $o/$tag/err.txt || exit 99
}
prof base1 MOFHIP_LIB=abvar/libmofhip_base.so
prof cur1 MOF_DUMMY=0
prof base2 MOFHIP_LIB=abvar/libmofhip_base.so
prof cur2 MOF_DUMMY=0
