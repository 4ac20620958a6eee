#!/bin/bash
# round-4 call 41: the final tree -- GPU suite, smoke, the default C3 line
export TMPDIR=/tmp
o=gpurun_out/r04c41
mkdir -p $o
S=tools/gpu_step.sh
$S 900 $o/gputests.log python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
$S 300 $o/smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 99
$S 600 $o/C3_default.json python3 bench.py || exit 99
