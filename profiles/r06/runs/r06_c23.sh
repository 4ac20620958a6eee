#!/bin/bash
# Round 6: C3 with the smoothed level-0 prolongator forced (MOF_AMG_SMOOTH=1):
# its iterations and where the time goes (the smoothed Galerkin product)
set -o pipefail
o=gpurun_out/r06c23; mkdir -p $o
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="--config C3 --steps 3 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 --legs none"
step c3_base python3 bench.py $B
MOF_AMG_SMOOTH=1 step c3_sa0 python3 bench.py $B
MOF_AMG_SMOOTH=1 MOF_VERBOSE=1 step prof_c3_sa0 rocprofv3 --kernel-trace --stats -d $o/prof_c3_sa0 -o run -- python3 bench.py $B
for f in $o/c3_*.out; do python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[1].split('/')[-1],l['value'],l['solver']['pcg_iterations_per_timestep'],l['ms_per_step'])" $f; done
