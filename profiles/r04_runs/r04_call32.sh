#!/bin/bash
# round-4 call 32: where symmetric reads stop paying -- R3 in plain RCM order
# (mirrored / plain lines 2.81) and S1s (1.53), forced symmetric vs plain
export TMPDIR=/tmp
o=gpurun_out/r04c32
mkdir -p $o
S=tools/gpu_step.sh
R="python3 bench.py --config R3 --steps 3 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0"
Q="python3 bench.py --config S1s --steps 30 --warmup 3 --no-cpu-baseline --parity-samples 0 --host-batches 0"
for r in 1 2; do
  MOF_WINDOW_SORT=0 MOF_SYM_READS=0 $S 300 $o/R3nows_plain_$r.json $R || exit 99
  MOF_WINDOW_SORT=0 MOF_SYM_READS=1 $S 300 $o/R3nows_sym_$r.json $R || exit 99
  MOF_SYM_READS=0 $S 300 $o/S1s_plain_$r.json $Q || exit 99
  MOF_SYM_READS=1 $S 300 $o/S1s_sym_$r.json $Q || exit 99
done
