#!/bin/bash
# S1s: boundary-row sweeps per side 0..4, twice each, on one box
set -o pipefail
D=gpurun_out/bswk
mkdir -p $D
for rep in 1 2; do
  for v in 0 1 2 3 4; do
    MOF_AMG_BSW=$v timeout -k 10 200 python3 -u bench.py --config S1s --no-cpu-baseline > $D/S1s_bsw${v}_r$rep.json 2> $D/e.err || exit 91
  done
done
