#!/bin/bash
# ab_multi.sh TAG "name:ENV=VAL ENV2=VAL" ... -- alternate bench.py runs of
# the default build without environment (base) and with each named set of
# runtime switches, one JSON line per run under gpurun_out/abm_TAG/.
# Extra bench arguments: AB_ARGS; runs per side: AB_REPS (2).
tag=$1; shift
out=gpurun_out/abm_$tag
mkdir -p $out
for rep in $(seq 1 ${AB_REPS:-2}); do
  for spec in "base:" "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    e=""; [ -n "$envs" ] && e="env $envs"
    $e timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 $AB_ARGS \
        > $out/${name}_$rep.json 2> $out/${name}_$rep.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "[ab] $name rc=$rc"; [ $rc -ne 1 ] && exit 99; fi
    python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[2],l['value'],l['roofline']['us_per_full_launch'],l['solver']['pcg_iterations_per_timestep'],l['solver']['ms_assembly_per_timestep'],l['solver']['ms_solve_per_timestep'])" $out/${name}_$rep.json $name
  done
done
