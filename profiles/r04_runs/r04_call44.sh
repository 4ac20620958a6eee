#!/bin/bash
# round-4 call 44: the final tree -- GPU suite, smoke, S1 / R3 lines
export TMPDIR=/tmp
o=gpurun_out/r04c44
mkdir -p $o
S=tools/gpu_step.sh
$S 900 $o/gputests.log python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
$S 300 $o/smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 99
$S 400 $o/S1.json python3 bench.py --config S1 --steps 4 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 400 $o/R3.json python3 bench.py --config R3 --steps 4 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
