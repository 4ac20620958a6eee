#!/bin/bash
# round-4 call 48: the final tree with the launch-grid guard -- GPU suite,
# smoke, short C3 / S1 / C5 lines (no grid past the bound)
export TMPDIR=/tmp
o=gpurun_out/r04c48
mkdir -p $o
S=tools/gpu_step.sh
$S 900 $o/gputests.log python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
$S 300 $o/smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 99
$S 300 $o/C3.json python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 300 $o/S1.json python3 bench.py --config S1 --steps 2 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 400 $o/C5.json python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
