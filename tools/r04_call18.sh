#!/bin/bash
# round-4 call 18: coarse-level symmetric reads (MOF_COARSE_SYM) -- tests,
# per-kernel times of both, C3 / S1 lines of both; the batch size on this build
export TMPDIR=/tmp
o=gpurun_out/r04c18
mkdir -p $o
S=tools/gpu_step.sh
$S 400 $o/tests.log python3 -u -m pytest tests/test_gpu_amg.py -v --timeout 200 --timeout-method thread -k "coarse_symmetric or galerkin" || exit 99
for v in 0 1; do
  mkdir -p $o/p_sym$v
  MOF_COARSE_SYM=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/p_sym$v -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/p_sym$v/bench.json 2> $o/p_sym$v/err.txt || exit 99
done
for v in 0 1 0 1; do
  MOF_COARSE_SYM=$v $S 300 $o/c3_s${v}_$RANDOM.json python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
done
for v in 0 1; do
  MOF_COARSE_SYM=$v $S 300 $o/S1_s${v}.json python3 bench.py --config S1 --steps 3 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
done
for b in 768 384; do
  $S 300 $o/c3_b${b}.json python3 bench.py --batch $b --steps 6 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
done
