#!/bin/bash
# round-4 call 4: HIP-graph replay (tests, small-job lines), fine-level
# damping 0.85 vs 0.7 on C3 / R3 / C2-mixed / S1, S1 damping diagnosis
o=gpurun_out/r04c4
mkdir -p $o
S=tools/gpu_step.sh
$S 300 $o/tests.log python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_graphs.py tests/test_gpu_fused.py tests/test_gpu_robust.py -k "graphs or fused or damped or accounting" || exit 99
$S 200 $o/C1_mixed_graphs.json python3 bench.py --config C1 --precision mixed --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
MOF_GRAPHS=0 $S 200 $o/C1_mixed_eager.json python3 bench.py --config C1 --precision mixed --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
$S 200 $o/S1s_mixed_graphs.json python3 bench.py --config S1s --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
MOF_AMG_OMEGA=0.7 $S 200 $o/S1s_mixed_graphs_om07.json python3 bench.py --config S1s --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
MOF_GRAPHS=0 MOF_AMG_OMEGA=0.7 $S 200 $o/S1s_mixed_eager_om07.json python3 bench.py --config S1s --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
for v in 0.85 0.7 0.6; do
  $S 300 $o/diag_S1_om$v.log python3 -u tools/diag_amg.py S1 4 MOF_AMG_OMEGA=$v || exit 99
done
for rep in 1 2; do
  $S 300 $o/c3_om085_$rep.json python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
  MOF_AMG_OMEGA=0.7 $S 300 $o/c3_om07_$rep.json python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
done
$S 300 $o/r3_om085.json python3 bench.py --config R3 --steps 3 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
MOF_AMG_OMEGA=0.7 $S 300 $o/r3_om07.json python3 bench.py --config R3 --steps 3 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
$S 300 $o/c2m_om085.json python3 bench.py --config C2 --precision mixed --steps 6 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
MOF_AMG_OMEGA=0.7 $S 300 $o/c2m_om07.json python3 bench.py --config C2 --precision mixed --steps 6 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
