#!/bin/bash
# batch_sweep.sh -- C3 bench at B = 512 / 768 / 1024, two alternating rounds, under gpurun_out/bsweep3/
mkdir -p gpurun_out/bsweep3
for r in 1 2; do for b in 512 768 1024; do
  timeout -k 10 300 python3 bench.py --batch $b --steps 8 --warmup 2 --no-cpu-baseline --parity-samples 0 --host-batches 0 > gpurun_out/bsweep3/b${b}_$r.json 2> gpurun_out/bsweep3/b${b}_$r.err || exit 99
  python3 -c "import json,sys;l=[json.loads(x) for x in open(sys.argv[1]) if x.startswith('{')][0];print(sys.argv[1],l['value'],l['roofline']['frac'],l['solver']['pcg_iterations_per_timestep'])" gpurun_out/bsweep3/b${b}_$r.json
done; done
