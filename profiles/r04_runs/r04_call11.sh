#!/bin/bash
# round-4 call 11: the reference's real workload end to end through the
# drop-in (tools/s3_end_to_end.py, fresh processes), then call 10's inner
# tolerance sweep
export TMPDIR=/tmp
o=gpurun_out/r04c11
mkdir -p $o
S=tools/gpu_step.sh
$S 200 $o/e2e_1.json python3 tools/s3_end_to_end.py S1s C1 || exit 99
$S 200 $o/e2e_2.json python3 tools/s3_end_to_end.py S1s C1 || exit 99
MOF_PRECISION=mixed $S 200 $o/e2e_mixed.json python3 tools/s3_end_to_end.py S1s C1 || exit 99
MOF_PRECISION=f64 $S 200 $o/e2e_f64.json python3 tools/s3_end_to_end.py S1s C1 || exit 99
bash tools/r04_call10.sh || exit 99
