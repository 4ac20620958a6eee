#!/bin/bash
# round-4 call 1: the full GPU suite (fused small-mesh solve, two lanes, 3-D
# residual), C1 / S1s lines eager vs fused, and the C3 A/B of the 3-D residual
# (MOF_RESIDUAL=rcn: the round-3 one), of the coarse Galerkin product by
# entry (MOF_GAL3_ENT=0: per position), of the 3-D a1 fold (MOF_ASM_G3=1) and
# of two batches in flight
o=gpurun_out/r04c1
mkdir -p $o
S=tools/gpu_step.sh
$S 600 $o/gputests.log python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread || exit 99
for cfg in C1 S1s; do
  $S 300 $o/bench_${cfg}_mixed.json python3 bench.py --config $cfg --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
  $S 300 $o/bench_${cfg}_f64_eager.json python3 bench.py --config $cfg --precision f64 --fused off --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
  $S 300 $o/bench_${cfg}_f64_fused.json python3 bench.py --config $cfg --precision f64 --fused on --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
done
for nq in 1 2 4; do
  MOF_FUSED_NQ=$nq $S 300 $o/bench_S1s_f64_fused_nq$nq.json python3 bench.py --config S1s --precision f64 --fused on --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 --parity-samples 0 || exit 99
done
for rep in 1 2; do
  $S 300 $o/c3_x3_$rep.json python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --parity-samples 1 --host-batches 0 || exit 99
  MOF_RESIDUAL=rcn $S 300 $o/c3_rcn_$rep.json python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
  MOF_ASM_G3=1 $S 300 $o/c3_g3_$rep.json python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --parity-samples 1 --host-batches 0 || exit 99
  MOF_GAL3_ENT=0 $S 300 $o/c3_gal3ns_$rep.json python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
  $S 300 $o/c3_l2_$rep.json python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 --lanes 2 || exit 99
done
