#!/bin/bash
# Round 6: XCD system-group size of the SpMV / level-0 sweeps / residual at
# B = 1536 (variant builds), rocprof kernel stats on C3
set -o pipefail
o=gpurun_out/r06c31; mkdir -p $o
L=$PWD/manifold-based-optical-flow-method_amd/mofhip
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
P="--config C3 --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 --legs none"
for v in base sp4 sp16 sm4 sm16 rs4 rs16 base2; do
  lib=""; case $v in base*) ;; *) lib=$L/libmofhip_$v.so;; esac
  MOFHIP_LIB=$lib step prof_c3_$v rocprofv3 --kernel-trace --stats -d $o/prof_c3_$v -o run -- python3 bench.py $P
done
for v in base sp4 sp16 sm4 sm16 rs4 rs16 base2; do echo $v; python3 tools/rocpd_stats.py $o/prof_c3_$v 40 | grep -E "spmv<float, false|post0|res0|residual|update"; done
