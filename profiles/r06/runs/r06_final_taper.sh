#!/bin/bash
# Round 6, final build (after the batch taper): GPU suite, smoke, the default bench line (as the
# driver runs it), and the C3 profile (kernel trace + FETCH / WRITE passes)
set -o pipefail
o=gpurun_out/r06fin3; mkdir -p $o
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
T=1000 step gputest python3 -u -m pytest tests -m gpu -x -q --timeout 800 --timeout-method thread
tail -2 $o/gputest.out
step smoke python3 -c "import __graft_entry__ as g; g.smoke()"
s=$(date +%s); T=500 step bench python3 bench.py; echo "bench wall $(( $(date +%s) - s ))s"
