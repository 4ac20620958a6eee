#!/bin/bash
# Round 6: the smoothed level-0 product from a bf16 slab (the sweep copy's
# blocks) against the fp32 slab: AMG tests, A/B lines (F3, S1, R3, C3 with
# level 0 smoothed), F3 kernel stats
set -o pipefail
o=gpurun_out/r06c32; mkdir -p $o
L=$PWD/manifold-based-optical-flow-method_amd/mofhip
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
T=700 step tests python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_amg.py
tail -1 $o/tests.out
B="--steps 4 --warmup 1 --no-cpu-baseline --parity-samples 2 --host-batches 0 --legs none"
for r in 1 2; do
  for c in F3 S1 R3; do
    step ${c}_new_$r python3 bench.py --config $c $B
    MOFHIP_LIB=$L/libmofhip_old.so step ${c}_old_$r python3 bench.py --config $c $B
  done
  MOF_AMG_SMOOTH=1 step C3sa_new_$r python3 bench.py --config C3 $B
  step C3_new_$r python3 bench.py --config C3 $B
done
for f in $o/[CFSR]*.out; do python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[1].split('/')[-1],l['value'],l['solver']['pcg_iterations_per_timestep'],l['ms_per_step'],l['parity']['max_abs_err'],l['solver']['recovered'])" $f; done
step prof_f3 rocprofv3 --kernel-trace --stats -d $o/prof_f3 -o run -- python3 bench.py --config F3 --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 --legs none
python3 tools/rocpd_stats.py $o/prof_f3 40 | grep -E "galerkin|a_slab"
