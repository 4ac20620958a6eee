#!/bin/bash
# round-4 call 2: the GPU suite on this build; the C3 default line (twice);
# the small jobs with their CPU baselines timed in full; S1s / S1 (the S1-like
# patches under the across-the-grid wave); R3
o=gpurun_out/r04c2
mkdir -p $o
S=tools/gpu_step.sh
$S 600 $o/gputests.log python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread || exit 99
$S 300 $o/c3_a.json python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
$S 400 $o/C1.json python3 bench.py --config C1 --steps 20 --warmup 2 || exit 99
$S 300 $o/S1s_mixed.json python3 bench.py --config S1s --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
$S 300 $o/S1s_f64.json python3 bench.py --config S1s --precision f64 --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
$S 400 $o/S1.json python3 bench.py --config S1 --steps 6 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
$S 400 $o/R3.json python3 bench.py --config R3 --steps 4 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 300 $o/c3_b.json python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
