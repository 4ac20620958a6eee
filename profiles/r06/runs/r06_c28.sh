#!/bin/bash
# Round 6: XCD system grouping of the smoothed transfers (kGrpRestr /
# kGrpProl, variant builds) on F3 and S1, kernel stats per variant
set -o pipefail
o=gpurun_out/r06c28; mkdir -p $o
L=$PWD/manifold-based-optical-flow-method_amd/mofhip
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
P="--steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 --legs none"
for v in base r8 r32 p8 p32; do
  lib=""; [ $v != base ] && lib=$L/libmofhip_$v.so
  MOFHIP_LIB=$lib step prof_f3_$v rocprofv3 --kernel-trace --stats -d $o/prof_f3_$v -o run -- python3 bench.py --config F3 $P
done
for v in base r8 r32 p8 p32; do echo $v; python3 tools/rocpd_stats.py $o/prof_f3_$v 40 | grep -E "restrict|prolong"; done
