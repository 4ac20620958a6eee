# F3 and C5 after the flat-level-0 rule (level 0 smoothed on folded meshes only where the finest aggregates are flat)
o=gpurun_out/r06c9; mkdir -p $o
S=tools/gpu_step.sh
MOF_VERBOSE=1 $S 400 $o/F3.json python3 bench.py --config F3 --steps 5 --warmup 1 --no-cpu-baseline --legs none --host-batches 0 || exit 99
MOF_VERBOSE=1 $S 400 $o/C5.json python3 bench.py --config C5 --batch 512 --steps 4 --warmup 1 --no-cpu-baseline --parity-samples 0 --legs none --host-batches 0 || exit 99
