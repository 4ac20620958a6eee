#!/bin/bash
# ab_bench.sh TAG VARIANT... -- alternate bench.py runs of the default build
# and each mofhip/libmofhip_VARIANT.so on one box (base, v1, v2, ..., base,
# v1, v2, ...), one JSON line per run under gpurun_out/ab_TAG/.
# Extra bench arguments: AB_ARGS; runs per build: AB_REPS (2).
tag=$1; shift
out=gpurun_out/ab_$tag
mkdir -p $out
for rep in $(seq 1 ${AB_REPS:-2}); do
  for v in base "$@"; do
    lib=""
    [ "$v" != base ] && lib=$PWD/manifold-based-optical-flow-method_amd/mofhip/libmofhip_$v.so
    MOFHIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 $AB_ARGS \
        > $out/${v}_$rep.json 2> $out/${v}_$rep.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "[ab] $v rc=$rc"; [ $rc -ne 1 ] && exit 99; fi
    python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[2],l['value'],l['roofline']['us_per_full_launch'],l['solver']['pcg_iterations_per_timestep'])" $out/${v}_$rep.json $v
  done
done
