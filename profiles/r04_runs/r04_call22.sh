#!/bin/bash
# round-4 call 22: the final default line (B = 1024, with its PMC entry
# committed), smoke, and the large configs at the default batch
export TMPDIR=/tmp
o=gpurun_out/r04c22
mkdir -p $o
S=tools/gpu_step.sh
$S 300 $o/smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 99
$S 600 $o/C3_default.json python3 bench.py || exit 99
$S 400 $o/S1.json python3 bench.py --config S1 --steps 3 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 400 $o/R3.json python3 bench.py --config R3 --steps 3 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 300 $o/C2.json python3 bench.py --config C2 --steps 6 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
