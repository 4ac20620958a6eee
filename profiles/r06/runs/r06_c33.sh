#!/bin/bash
# Round 6: the bf16 slab for the smoothed level-0 product on regular closed
# meshes only (F3; C3 with MOF_AMG_SMOOTH=1) against the fp32 slab; S1 / R3
# keep the fp32 slab (V hashes against the previous build)
set -o pipefail
o=gpurun_out/r06c33; mkdir -p $o
L=$PWD/manifold-based-optical-flow-method_amd/mofhip
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
T=700 step tests python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_amg.py tests/test_gpu_robust.py -k "f3 or folded or smoothed or slab"
tail -1 $o/tests.out
step vh_s1m_new python3 tools/vhash.py S1m 9
MOFHIP_LIB=$L/libmofhip_old.so step vh_s1m_old python3 tools/vhash.py S1m 9
step vh_r3_new python3 tools/vhash.py R3 9
MOFHIP_LIB=$L/libmofhip_old.so step vh_r3_old python3 tools/vhash.py R3 9
cat $o/vh_*.out
B="--steps 4 --warmup 1 --no-cpu-baseline --parity-samples 2 --host-batches 0 --legs none"
for r in 1 2; do
  step F3_new_$r python3 bench.py --config F3 $B
  MOFHIP_LIB=$L/libmofhip_old.so step F3_old_$r python3 bench.py --config F3 $B
  MOF_AMG_SMOOTH=1 step C3sa_new_$r python3 bench.py --config C3 $B
  MOF_AMG_SMOOTH=1 MOFHIP_LIB=$L/libmofhip_old.so step C3sa_old_$r python3 bench.py --config C3 $B
done
for f in $o/[CF]*.out; do python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[1].split('/')[-1],l['value'],l['solver']['pcg_iterations_per_timestep'],l['ms_per_step'],l['parity']['max_abs_err'],l['solver']['recovered'])" $f; done
