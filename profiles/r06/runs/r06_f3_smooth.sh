# F3 with the level-0 smoothed prolongator forced on, against the default (tentative level 0)
set -e
mkdir -p gpurun_out/r06c4
run() { name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config F3 --legs none --no-cpu-baseline --steps 5 --warmup 1 --host-batches 0 --parity-samples 0 > gpurun_out/r06c4/$name.json 2> gpurun_out/r06c4/$name.err
}
run f3_auto MOF_VERBOSE=1
run f3_sa0 MOF_VERBOSE=1 MOF_AMG_SMOOTH=1
run f3_auto_b MOF_VERBOSE=1
run f3_sa0_b MOF_VERBOSE=1 MOF_AMG_SMOOTH=1
