#!/bin/bash
# round-4 call 36: restriction sums by (coarse node, system) instead of by
# coarse node (bit-identical), with 4 / 8 systems per smoothed-P workgroup
# and prolongation thread -- V hashes (S1s: smoothed P; C2 mesh: tentative
# P) and per-kernel times on S1 and C3 against the committed build
export TMPDIR=/tmp
o=gpurun_out/r04c36
mkdir -p $o
for v in base new n8 n48; do
  if [ $v = new ]; then L=""; else L="MOFHIP_LIB=abvar/libmofhip_$v.so"; fi
  env $L timeout -k 10 120 python3 tools/vhash.py S1s 98 > $o/vhash_S1s_$v.json 2> $o/vhash_S1s_$v.err || exit 99
  env $L timeout -k 10 120 python3 tools/vhash.py S1s 98 40 > $o/vhash_S1s40_$v.json 2> $o/vhash_S1s40_$v.err || exit 99
  env $L timeout -k 10 120 python3 tools/vhash.py C2 41 > $o/vhash_C2_$v.json 2> $o/vhash_C2_$v.err || exit 99
done
prof() {  # tag config env...
  local tag=$1 cfg=$2; shift 2
  mkdir -p $o/$tag
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$tag -o run -- \
      python3 bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/$tag/bench.json 2> $o/$tag/err.txt || exit 99
}
for v in base new n8 n48; do
  if [ $v = new ]; then L="MOF_DUMMY=0"; else L="MOFHIP_LIB=abvar/libmofhip_$v.so"; fi
  prof S1_$v S1 $L
  prof C3_$v C3 $L
done
