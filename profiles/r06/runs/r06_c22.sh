#!/bin/bash
# Round 6: the default bench line (C3 + F3 / S1s / S1 legs) as the driver runs it, and smoke
set -o pipefail
o=gpurun_out/r06c22; mkdir -p $o
s=$(date +%s)
timeout -k 10 500 python3 bench.py > $o/bench_default.json 2> $o/bench_default.err; rc=$?
echo "[bench] rc=$rc wall=$(( $(date +%s) - s ))s"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.out 2>&1; rc=$?
echo "[smoke] rc=$rc"; exit $rc
