# level >= 1 sweeps (k_res3 / k_post3) in the XCD-aware grid order (variant
# builds, MOF_EXP_L1XCD = G systems per group) against the system-major grid;
# C3 and S1, alternating on one box
o=gpurun_out/r06c10; mkdir -p $o
S=tools/gpu_step.sh
L=manifold-based-optical-flow-method_amd/mofhip
B="python3 bench.py --legs none --no-cpu-baseline --parity-samples 0 --host-batches 0 --steps 10 --warmup 2"
for r in 1 2; do
  $S 300 $o/C3_base_$r.json $B || exit 99
  MOFHIP_LIB=$L/libmofhip_l1x8.so $S 300 $o/C3_x8_$r.json $B || exit 99
  MOFHIP_LIB=$L/libmofhip_l1x32.so $S 300 $o/C3_x32_$r.json $B || exit 99
done
$S 300 $o/S1_base.json $B --config S1 --steps 3 --warmup 1 || exit 99
MOFHIP_LIB=$L/libmofhip_l1x8.so $S 300 $o/S1_x8.json $B --config S1 --steps 3 --warmup 1 || exit 99
