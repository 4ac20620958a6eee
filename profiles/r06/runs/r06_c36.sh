#!/bin/bash
# Round 6: tapered first / last batches of host-pointer jobs: host-path GPU
# tests, then the C3 line's host_io (4 batches) and --io host against the
# previous build, alternating
set -o pipefail
o=gpurun_out/r06c36; mkdir -p $o
L=$PWD/manifold-based-optical-flow-method_amd/mofhip
step() { local n=$1; shift; timeout -k 10 ${T:-300} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
T=600 step tests python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_robust.py -k "host_pipeline or dropin" tests/test_gpu_parity.py
tail -1 $o/tests.out
B="--steps 6 --warmup 1 --no-cpu-baseline --parity-samples 0 --legs none"
for r in 1 2; do
  step c3_new_$r python3 bench.py $B
  MOFHIP_LIB=$L/libmofhip_old.so step c3_old_$r python3 bench.py $B
  step c3io_new_$r python3 bench.py --io host --steps 6 --warmup 1 --no-cpu-baseline --parity-samples 0
  MOFHIP_LIB=$L/libmofhip_old.so step c3io_old_$r python3 bench.py --io host --steps 6 --warmup 1 --no-cpu-baseline --parity-samples 0
done
for f in $o/c3*.out; do python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[1].split('/')[-1],l['value'],(l.get('host_io') or {}).get('value'),l['solver']['recovered'])" $f; done
