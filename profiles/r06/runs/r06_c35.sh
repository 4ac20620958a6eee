#!/bin/bash
# Round 6: C3 with level 0 smoothed and level 1 tentative (variant build) on
# the final build (symmetric products, bf16 slab, transfer grouping) against
# the default tentative hierarchy
set -o pipefail
o=gpurun_out/r06c35; mkdir -p $o
L=$PWD/manifold-based-optical-flow-method_amd/mofhip
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="--config C3 --steps 4 --warmup 1 --no-cpu-baseline --parity-samples 2 --host-batches 0 --legs none"
for r in 1 2 3; do
  step C3_def_$r python3 bench.py $B
  MOF_AMG_SMOOTH=1 MOFHIP_LIB=$L/libmofhip_sa0only.so step C3_sa0_$r python3 bench.py $B
done
for f in $o/C3*.out; do python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[1].split('/')[-1],l['value'],l['solver']['pcg_iterations_per_timestep'],l['ms_per_step'],l['parity']['max_abs_err'],l['solver']['recovered'])" $f; done
