#!/bin/bash
# Round 6: the bf16 slab on the irregular closed mesh R3 too (variant build)
set -o pipefail
o=gpurun_out/r06c34; mkdir -p $o
L=$PWD/manifold-based-optical-flow-method_amd/mofhip
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="--steps 4 --warmup 1 --no-cpu-baseline --parity-samples 2 --host-batches 0 --legs none"
for r in 1 2; do
  step R3_base_$r python3 bench.py --config R3 $B
  MOFHIP_LIB=$L/libmofhip_slabc.so step R3_slabh_$r python3 bench.py --config R3 $B
done
for f in $o/R3*.out; do python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[1].split('/')[-1],l['value'],l['solver']['pcg_iterations_per_timestep'],l['ms_per_step'],l['parity']['max_abs_err'],l['solver']['recovered'])" $f; done
