#!/bin/bash
# k_bsweep with the per-slot ring-position table: bit-identity proxies
# (S1s / S1 parity errors and iterations) and S1 with the sweeps forced on
set -o pipefail
D=gpurun_out/bsw3
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_amg.py -k "open_patch" -x -v --timeout 120 --timeout-method thread > $D/t.log 2>&1 || exit 90
timeout -k 10 200 python3 -u bench.py --config S1s --no-cpu-baseline > $D/S1s_auto.json 2> $D/e1.err || exit 91
for v in 2 0 2 0; do
  MOF_AMG_BSW=$v timeout -k 10 240 python3 -u bench.py --config S1 --no-cpu-baseline > $D/S1_bsw${v}_$RANDOM.json 2> $D/e2.err || exit 92
done
