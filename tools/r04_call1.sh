#!/bin/bash
# round-4 call 1: the fused small-mesh solve (tests, C1 / S1s lines eager vs
# fused), two batches in flight (tools/streams2.py) and the coarse Galerkin
# product by gather entry (libmofhip_gal3.so) against the default build
o=gpurun_out/r04c1
mkdir -p $o
S=tools/gpu_step.sh
$S 300 $o/fused_tests.log python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused.py || exit 99
for cfg in C1 S1s; do
  $S 300 $o/bench_${cfg}_mixed.json python3 bench.py --config $cfg --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
  $S 300 $o/bench_${cfg}_f64_eager.json python3 bench.py --config $cfg --precision f64 --fused off --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
  $S 300 $o/bench_${cfg}_f64_fused.json python3 bench.py --config $cfg --precision f64 --fused on --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
done
$S 400 $o/streams_512.jsonl python3 -u tools/streams2.py C3 512 6 || exit 99
$S 400 $o/streams_256.jsonl python3 -u tools/streams2.py C3 256 12 || exit 99
AB_REPS=2 bash tools/ab_bench.sh r04gal3 gal3 || exit 99
