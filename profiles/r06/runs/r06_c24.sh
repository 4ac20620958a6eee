#!/bin/bash
# Round 6: C3 with the smoothed level-0 prolongator and a tentative level 1
# (variant build) against the default and against both levels smoothed
set -o pipefail
o=gpurun_out/r06c24; mkdir -p $o
L=$PWD/manifold-based-optical-flow-method_amd/mofhip
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="--config C3 --steps 4 --warmup 1 --no-cpu-baseline --parity-samples 2 --host-batches 0 --legs none"
for r in 1 2; do
step c3_base_$r python3 bench.py $B
MOF_AMG_SMOOTH=1 step c3_sa01_$r python3 bench.py $B
MOF_AMG_SMOOTH=1 MOFHIP_LIB=$L/libmofhip_sa0only.so step c3_sa0_$r python3 bench.py $B
done
MOF_AMG_SMOOTH=1 MOFHIP_LIB=$L/libmofhip_sa0only.so step prof_c3_sa0 rocprofv3 --kernel-trace --stats -d $o/prof_c3_sa0 -o run -- python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 --legs none
for f in $o/c3_*.out; do python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[1].split('/')[-1],l['value'],l['solver']['pcg_iterations_per_timestep'],l['ms_per_step'],l['parity']['max_abs_err'])" $f; done
