#!/bin/bash
# round-4 call 8: the 3-D system-major residual (k_residual_x3sm) -- agreement
# tests with k_residual_rcn, C3 lines with MOF_RES_SM=0 / 1 on one box,
# per-kernel times of both (rocprof stats)
export TMPDIR=/tmp
o=gpurun_out/r04c8
mkdir -p $o
S=tools/gpu_step.sh
$S 400 $o/tests_sm.log python3 -u -m pytest tests/test_gpu_residual_sm.py -v --timeout 200 --timeout-method thread || exit 99
grep -q "6 passed" $o/tests_sm.log || exit 98
for v in 0 1; do
  mkdir -p $o/p_sm$v
  MOF_RES_SM=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/p_sm$v -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/p_sm$v/bench.json 2> $o/p_sm$v/err.txt || exit 99
done
for v in 0 1 0 1; do
  MOF_RES_SM=$v $S 300 $o/c3_sm${v}_$RANDOM.json python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
done
