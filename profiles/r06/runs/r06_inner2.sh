# deeper first inner solves on the large smoothed-hierarchy meshes, second sweep
o=gpurun_out/r06c12; mkdir -p $o
S=tools/gpu_step.sh
B="python3 bench.py --legs none --no-cpu-baseline --parity-samples 2 --host-batches 0 --steps 3 --warmup 1"
for t in 1e-7 3e-8 3e-7; do
  MOF_VERBOSE=1 $S 300 $o/S1_$t.json $B --config S1 --inner-rtol $t || exit 99
done
MOF_VERBOSE=1 $S 300 $o/S1_1e-5.json $B --config S1 --inner-rtol 1e-5 || exit 99
for t in 3e-7 1e-7; do
  MOF_VERBOSE=1 $S 300 $o/R3_$t.json $B --config R3 --inner-rtol $t || exit 99
done
for t in 1e-5 3e-7 1e-7; do
  MOF_VERBOSE=1 $S 300 $o/S1m_$t.json $B --config S1m --inner-rtol $t || exit 99
done
