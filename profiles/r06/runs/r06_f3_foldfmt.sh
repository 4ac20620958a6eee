# F3: level-0 smoothed prolongator with the regular-mesh formats (bf16 z,
# in-place bf16 corrected iterate, coarse damping 1.1; variant build
# libmofhip_foldfmt.so) against the default and against plain SA0
set -e
mkdir -p gpurun_out/r06c5
run() { name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config F3 --legs none --no-cpu-baseline --steps 5 --warmup 1 --host-batches 0 --parity-samples 2 > gpurun_out/r06c5/$name.json 2> gpurun_out/r06c5/$name.err
}
V=manifold-based-optical-flow-method_amd/mofhip/libmofhip_foldfmt.so
run auto_1 MOF_VERBOSE=1
run ffmt_1 MOF_VERBOSE=1 MOF_AMG_SMOOTH=1 MOFHIP_LIB=$V
run sa0_1 MOF_VERBOSE=1 MOF_AMG_SMOOTH=1
run auto_2 MOF_VERBOSE=1
run ffmt_2 MOF_VERBOSE=1 MOF_AMG_SMOOTH=1 MOFHIP_LIB=$V
