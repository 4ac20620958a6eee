#!/bin/bash
# round-4 call 5b: S1 (160k open patch) with open surfaces kept off the bf16
# iterates; variants
o=gpurun_out/r04c5b
mkdir -p $o
S=tools/gpu_step.sh
$S 300 $o/diag_S1_default.log python3 -u tools/diag_amg.py S1 4 || exit 99
$S 300 $o/diag_S1_xbf16.log python3 -u tools/diag_amg.py S1 4 MOF_X_BF16=1 || exit 99
$S 300 $o/diag_S1_om085.log python3 -u tools/diag_amg.py S1 4 MOF_AMG_OMEGA=0.85 || exit 99
$S 300 $o/diag_S1_smooth.log python3 -u tools/diag_amg.py S1 4 MOF_AMG_SMOOTH=1 || exit 99
$S 400 $o/S1.json python3 bench.py --config S1 --steps 4 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 300 $o/S1s.json python3 bench.py --config S1s --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
