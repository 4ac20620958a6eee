#!/bin/bash
# round-4 call 15: host pipeline tests (ring and direct copies); the
# end-to-end small jobs with direct pageable copies
export TMPDIR=/tmp
o=gpurun_out/r04c15
mkdir -p $o
S=tools/gpu_step.sh
$S 400 $o/tests.log python3 -u -m pytest tests/test_gpu_robust.py -k "host_pipeline" -v --timeout 200 --timeout-method thread || exit 99
MOF_HOSTIO_VERBOSE=1 $S 200 $o/e2e_1.json python3 tools/s3_end_to_end.py S1s C1 || exit 99
$S 200 $o/e2e_2.json python3 tools/s3_end_to_end.py S1s C1 || exit 99
$S 300 $o/C3_host.json python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --parity-samples 0 || exit 99
