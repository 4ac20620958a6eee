#!/bin/bash
# Round 6: the new open-surface defaults (sweeps everywhere, coarse levels
# smoothed): their GPU tests, the open-patch benches with parity
set -o pipefail
o=gpurun_out/r06bsw3; mkdir -p $o
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
T=900 step tests python3 -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_gpu_amg.py -k "boundary_sweeps or pinwheel or open" tests/test_gpu_robust.py::test_s1_full_size_default_vs_spsolve tests/test_gpu_robust.py::test_s1s_dropin_defaults_vs_spsolve tests/test_gpu_robust.py::test_damped_multigrid_recovery_on_pinwheel_patch
tail -15 $o/tests.out
for c in S1 S1m; do step $c python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --host-batches 2 --legs none; done
step S1s python3 bench.py --config S1s --steps 20 --warmup 2 --no-cpu-baseline --host-batches 2 --legs none
for f in $o/S1*.out; do python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[1].split('/')[-1],l['value'],(l.get('host_io') or {}).get('value'),l['solver']['pcg_iterations_per_timestep'],l['solver'].get('recovered'),l['parity']['max_abs_err'],l['roofline']['frac'],l.get('defect'))" $f; done
