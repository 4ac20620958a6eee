#!/bin/bash
# round-4 call 47: the final tree (by-entry Galerkin only where its grid fits
# 2^32 work-items) -- GPU suite, smoke, V hashes, the default C3 line
export TMPDIR=/tmp
o=gpurun_out/r04c47
mkdir -p $o
S=tools/gpu_step.sh
$S 900 $o/gputests.log python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
$S 300 $o/smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 99
$S 120 $o/vhash_C2.json python3 tools/vhash.py C2 41 || exit 99
$S 200 $o/vhash_S1.json python3 tools/vhash.py S1 1025 || exit 99
$S 600 $o/C3_default.json python3 bench.py || exit 99
