#!/bin/bash
# round-4 call 24: the residual with the row's incidence entries preloaded (162 VGPRs, 3 waves) against
# the same build without (libmofhip_base.so: 128 VGPRs, 4 waves) -- kernel
# stats and C3 lines, one box
export TMPDIR=/tmp
o=gpurun_out/r04c24
mkdir -p $o
S=tools/gpu_step.sh
BASE=$PWD/manifold-based-optical-flow-method_amd/mofhip/libmofhip_base.so
for v in base new; do
  mkdir -p $o/p_$v
  lib=""; [ $v = base ] && lib=$BASE
  MOFHIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/p_$v -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/p_$v/bench.json 2> $o/p_$v/err.txt || exit 99
done
for v in base new base new; do
  lib=""; [ $v = base ] && lib=$BASE
  MOFHIP_LIB=$lib $S 300 $o/c3_${v}_$RANDOM.json python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
done
