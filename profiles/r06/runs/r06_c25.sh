#!/bin/bash
# Round 6: the smoothed level-0 Galerkin product from LDS-staged blocks:
# bits against the slab kernel, then the smoothed-hierarchy meshes
set -o pipefail
o=gpurun_out/r06c25; mkdir -p $o
L=$PWD/manifold-based-optical-flow-method_amd/mofhip
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step vh_f3_new python3 tools/vhash.py F3 9
MOFHIP_LIB=$L/libmofhip_old.so step vh_f3_old python3 tools/vhash.py F3 9
step vh_s1m_new python3 tools/vhash.py S1m 9
MOFHIP_LIB=$L/libmofhip_old.so step vh_s1m_old python3 tools/vhash.py S1m 9
step vh_r3_new python3 tools/vhash.py R3 9
MOFHIP_LIB=$L/libmofhip_old.so step vh_r3_old python3 tools/vhash.py R3 9
MOF_AMG_SMOOTH=1 step vh_c3_new python3 tools/vhash.py C3 9
MOF_AMG_SMOOTH=1 MOFHIP_LIB=$L/libmofhip_old.so step vh_c3_old python3 tools/vhash.py C3 9
cat $o/vh_*.out
B="--steps 4 --warmup 1 --no-cpu-baseline --parity-samples 2 --host-batches 0 --legs none"
for c in F3 S1 R3; do
  step ${c}_new python3 bench.py --config $c $B
  MOFHIP_LIB=$L/libmofhip_old.so step ${c}_old python3 bench.py --config $c $B
done
step C3_base python3 bench.py --config C3 $B
MOF_AMG_SMOOTH=1 MOFHIP_LIB=$L/libmofhip_sa0only.so step C3_sa0 python3 bench.py --config C3 $B
step C3_base2 python3 bench.py --config C3 $B
MOF_AMG_SMOOTH=1 MOFHIP_LIB=$L/libmofhip_sa0only.so step C3_sa0_2 python3 bench.py --config C3 $B
for f in $o/[FSRC]*.out; do python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[1].split('/')[-1],l['value'],l['solver']['pcg_iterations_per_timestep'],l['ms_per_step'],l['parity']['max_abs_err'])" $f; done
step prof_f3 rocprofv3 --kernel-trace --stats -d $o/prof_f3 -o run -- python3 bench.py --config F3 --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 --legs none
