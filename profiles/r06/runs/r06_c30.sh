#!/bin/bash
# Round 6: systems per workgroup / thread of the smoothed transfers (kNSR,
# kNSP) and the XCD-aware grid for the level >= 1 sweeps, variant builds;
# rocprof kernel stats on F3 / C3
set -o pipefail
o=gpurun_out/r06c30; mkdir -p $o
L=$PWD/manifold-based-optical-flow-method_amd/mofhip
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
P="--steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 --legs none"
for v in base nsr4 nsr16 nsp8 l1x; do
  lib=""; [ $v != base ] && lib=$L/libmofhip_$v.so
  MOFHIP_LIB=$lib step prof_f3_$v rocprofv3 --kernel-trace --stats -d $o/prof_f3_$v -o run -- python3 bench.py --config F3 $P
done
for v in base l1x; do
  lib=""; [ $v != base ] && lib=$L/libmofhip_$v.so
  MOFHIP_LIB=$lib step prof_c3_$v rocprofv3 --kernel-trace --stats -d $o/prof_c3_$v -o run -- python3 bench.py --config C3 $P
done
for d in $o/prof_*; do [ -d $d ] || continue; echo $(basename $d); python3 tools/rocpd_stats.py $d 40 | grep -E "restrict|prolong|res3|post3"; done
