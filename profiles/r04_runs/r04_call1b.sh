#!/bin/bash
# round-4 call 1b: the GPU suite (after the decomposed test hook fix), the
# S1s multigrid failure (variants), per-kernel times of the setup-kernel
# variants (rocprof stats), two lanes at B = 256
export TMPDIR=/tmp
o=gpurun_out/r04c1b
mkdir -p $o
S=tools/gpu_step.sh
$S 600 $o/gputests.log python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread || exit 99
for v in "" MOF_AMG_SMOOTH=0 MOF_X_BF16=0 MOF_X_BF16=1 MOF_WINDOW_SORT=0 MOF_AMG_OMEGA=0.7 MOF_AMG_OMEGA1=0.9 MOF_PCG_STALL=0; do
  tag=$(echo "d_$v" | tr '=' '_')
  $S 200 $o/diag_S1s_$tag.log python3 -u tools/diag_amg.py S1s 8 $v || exit 99
done
for v in MOF_RESIDUAL=rcn "MOF_RESIDUAL=rcn MOF_ASM_G3=1" MOF_RESIDUAL=x3 "MOF_RESIDUAL=rcn MOF_GAL3_ENT=0"; do
  tag=$(echo "p_$v" | tr '= ' '__')
  mkdir -p $o/$tag
  env $v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$tag -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/$tag/bench.json 2> $o/$tag/err.txt || exit 99
done
$S 300 $o/c3_b256_l1.json python3 bench.py --batch 256 --steps 12 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 || exit 99
$S 300 $o/c3_b256_l2.json python3 bench.py --batch 256 --steps 12 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 --lanes 2 || exit 99
