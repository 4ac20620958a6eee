#!/bin/bash
# round-4 call 12: the GPU suite on this build; the end-to-end small jobs with
# the job-sized staging ring (setup steps under MOF_HOSTIO_VERBOSE); S1 / R3 /
# S1s lines with the deeper first inner solve on smoothed hierarchies; C3
export TMPDIR=/tmp
o=gpurun_out/r04c12
mkdir -p $o
S=tools/gpu_step.sh
$S 900 $o/gputests.log python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
MOF_HOSTIO_VERBOSE=1 $S 200 $o/e2e_1.json python3 tools/s3_end_to_end.py S1s C1 || exit 99
$S 200 $o/e2e_2.json python3 tools/s3_end_to_end.py S1s C1 || exit 99
$S 300 $o/S1.json python3 bench.py --config S1 --steps 4 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 300 $o/R3.json python3 bench.py --config R3 --steps 4 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 300 $o/S1s.json python3 bench.py --config S1s --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
$S 300 $o/C3.json python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
