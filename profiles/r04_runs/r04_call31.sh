#!/bin/bash
# round-4 call 31: the S1-like patch (160,801 vertices) with symmetric reads
# forced and with the window sort off, against its defaults, interleaved
export TMPDIR=/tmp
o=gpurun_out/r04c31
mkdir -p $o
S=tools/gpu_step.sh
B="python3 bench.py --config S1 --steps 3 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0"
for r in 1 2; do
  $S 300 $o/S1_def_$r.json $B || exit 99
  MOF_SYM_READS=1 $S 300 $o/S1_sym_$r.json $B || exit 99
  MOF_WINDOW_SORT=0 $S 300 $o/S1_nows_$r.json $B || exit 99
done
