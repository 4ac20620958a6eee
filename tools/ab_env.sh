#!/bin/bash
# ab_env.sh TAG "ENV=VAL ..." -- alternate bench.py runs of the default build
# without and with the given environment (runtime A/B switches), one JSON line
# per run under gpurun_out/abenv_TAG/. Extra bench arguments: AB_ARGS; runs
# per side: AB_REPS (2).
tag=$1; envs=$2
out=gpurun_out/abenv_$tag
mkdir -p $out
for rep in $(seq 1 ${AB_REPS:-2}); do
  for side in base var; do
    if [ $side = var ]; then e="env $envs"; else e=""; fi
    $e timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 $AB_ARGS \
        > $out/${side}_$rep.json 2> $out/${side}_$rep.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "[ab] $side rc=$rc"; [ $rc -ne 1 ] && exit 99; fi
    python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[2],l['value'],l['roofline']['us_per_full_launch'],l['solver']['pcg_iterations_per_timestep'],l['solver']['ms_assembly_per_timestep'],l['solver']['ms_solve_per_timestep'])" $out/${side}_$rep.json $side
  done
done
