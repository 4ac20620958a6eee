#!/bin/bash
# Round 6: Galerkin products over the diagonal and upper coarse blocks only,
# each lower block written by its upper twin (st_pair): AMG GPU tests, A/B lines
set -o pipefail
o=gpurun_out/r06c27; mkdir -p $o
L=$PWD/manifold-based-optical-flow-method_amd/mofhip
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
T=700 step tests python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_amg.py tests/test_gpu_parity.py
tail -2 $o/tests.out
B="--steps 4 --warmup 1 --no-cpu-baseline --parity-samples 2 --host-batches 0 --legs none"
for r in 1 2; do for c in C3 F3 S1 R3; do
  step ${c}_new_$r python3 bench.py --config $c $B
  MOFHIP_LIB=$L/libmofhip_old.so step ${c}_old_$r python3 bench.py --config $c $B
done; done
for f in $o/[CFSR]*.out; do python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[1].split('/')[-1],l['value'],l['solver']['pcg_iterations_per_timestep'],l['ms_per_step'],l['parity']['max_abs_err'],l['solver']['recovered'])" $f; done
step prof_c3 rocprofv3 --kernel-trace --stats -d $o/prof_c3 -o run -- python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 --legs none
step prof_f3 rocprofv3 --kernel-trace --stats -d $o/prof_f3 -o run -- python3 bench.py --config F3 --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 --legs none
