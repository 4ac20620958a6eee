# first inner tolerance on the large smoothed-hierarchy meshes (S1, R3) with
# the error control in place: 1e-5 (the default since round 4) against
# deeper first steps; one box
o=gpurun_out/r06c11; mkdir -p $o
S=tools/gpu_step.sh
B="python3 bench.py --legs none --no-cpu-baseline --parity-samples 2 --host-batches 0 --steps 3 --warmup 1"
for t in 1e-5 3e-6 1e-6 3e-7; do
  MOF_VERBOSE=1 $S 300 $o/S1_$t.json $B --config S1 --inner-rtol $t || exit 99
done
for t in 1e-5 1e-6; do
  MOF_VERBOSE=1 $S 300 $o/R3_$t.json $B --config R3 --inner-rtol $t || exit 99
done
MOF_VERBOSE=1 $S 300 $o/S1_1e-5_b.json $B --config S1 --inner-rtol 1e-5 || exit 99
