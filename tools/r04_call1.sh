#!/bin/bash
# round-4 call 1: the fused small-mesh solve (tests, C1 / S1s lines eager vs
# fused) and two batches in flight (MOF_TWO_LANES: tests, C3 A/B)
o=gpurun_out/r04c1
mkdir -p $o
S=tools/gpu_step.sh
$S 400 $o/tests.log python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_lanes.py || exit 99
for cfg in C1 S1s; do
  $S 300 $o/bench_${cfg}_mixed.json python3 bench.py --config $cfg --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
  $S 300 $o/bench_${cfg}_f64_eager.json python3 bench.py --config $cfg --precision f64 --fused off --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
  $S 300 $o/bench_${cfg}_f64_fused.json python3 bench.py --config $cfg --precision f64 --fused on --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
done
for rep in 1 2; do
  $S 300 $o/c3_l1_$rep.json python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
  $S 300 $o/c3_l2_$rep.json python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 --lanes 2 || exit 99
  $S 300 $o/c3_l2b256_$rep.json python3 bench.py --steps 16 --warmup 2 --batch 256 --no-cpu-baseline --parity-samples 0 --host-batches 0 --lanes 2 || exit 99
done
