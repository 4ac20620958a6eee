set -e
mkdir -p gpurun_out/r06c3
run() { # name env...
  name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config S1 --legs none --no-cpu-baseline --steps 2 --warmup 1 --allow-recovery --host-batches 0 --parity-samples 0 > gpurun_out/r06c3/$name.json 2> gpurun_out/r06c3/$name.err
}
run base MOF_VERBOSE=1
run w_om1_090 MOF_VERBOSE=1 MOF_AMG_W=1 MOF_AMG_OMEGA=0.7,0.9
run w_om1_080 MOF_VERBOSE=1 MOF_AMG_W=1 MOF_AMG_OMEGA=0.7,0.8
run v_om1_090 MOF_VERBOSE=1 MOF_AMG_OMEGA=0.7,0.9
run w_om1_105 MOF_VERBOSE=1 MOF_AMG_W=1
