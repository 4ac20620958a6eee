#!/bin/bash
# Round 6: GPU suite on the new open-surface defaults; first inner tolerance
# of the open patches under them
set -o pipefail
o=gpurun_out/r06c20; mkdir -p $o
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
T=1100 step gputest python3 -u -m pytest tests -m gpu -x -q --timeout 800 --timeout-method thread
tail -3 $o/gputest.out
B="--legs none --no-cpu-baseline --parity-samples 2 --host-batches 0 --steps 3 --warmup 1"
for c in S1 S1m; do for t in 1e-5 3e-6 1e-6 3e-7; do step ${c}_$t python3 bench.py --config $c --inner-rtol $t $B; done; done
for f in $o/S1*.out; do python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[1].split('/')[-1],l['value'],l['solver']['pcg_iterations_per_timestep'],l['solver'].get('recovered'),l['parity']['max_abs_err'],l.get('defect'))" $f; done
