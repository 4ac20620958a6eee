#!/bin/bash
# round-4 call 13: the residual's incidence-geometry planes -- bit-identity
# tests, per-kernel times with the planes and with the per-lane gathers
# (MOF_RES_GATHER=1), C3 lines of both
export TMPDIR=/tmp
o=gpurun_out/r04c13
mkdir -p $o
S=tools/gpu_step.sh
$S 400 $o/tests.log python3 -u -m pytest tests/test_gpu_residual_geometry.py -v --timeout 200 --timeout-method thread || exit 99
grep -q "5 passed" $o/tests.log || exit 98
for v in 1 0; do
  mkdir -p $o/p_gather$v
  MOF_RES_GATHER=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/p_gather$v -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/p_gather$v/bench.json 2> $o/p_gather$v/err.txt || exit 99
done
for v in 1 0 1 0; do
  MOF_RES_GATHER=$v $S 300 $o/c3_g${v}_$RANDOM.json python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
done
