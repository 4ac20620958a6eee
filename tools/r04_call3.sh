#!/bin/bash
# round-4 call 3: fine-level damping on the S1-like patches (diag, variants),
# launch-latency probe
o=gpurun_out/r04c3
mkdir -p $o
S=tools/gpu_step.sh
for cfg in S1s S1; do
  for v in MOF_AMG_OMEGA=0.85 MOF_AMG_OMEGA=0.7 MOF_AMG_OMEGA=0.6 MOF_AMG_OMEGA=0.5 "MOF_AMG_OMEGA=0.6 MOF_AMG_SMOOTH=0" "MOF_AMG_OMEGA=0.6 MOF_AMG_OMEGA1=0.9" "MOF_AMG_OMEGA=0.6 MOF_X_BF16=1"; do
    tag=$(echo "$v" | tr '= ' '__')
    $S 300 $o/diag_${cfg}_$tag.log python3 -u tools/diag_amg.py $cfg 8 $v || exit 99
  done
done
$S 120 $o/graph_probe.json python3 tools/graph_probe.py 400 || exit 99
