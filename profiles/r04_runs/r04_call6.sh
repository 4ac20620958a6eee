#!/bin/bash
# round-4 call 6: the GPU suite and the S1 lines on this build; counters of the setup kernels before (the round-3 library,
# libmofhip_r3.so) and after (this build): SQ issue / wait shares, FETCH_SIZE,
# WRITE_SIZE, each pass its own run; then the final profile of the default
# line (kernel trace + stats, separate FETCH / WRITE passes)
export TMPDIR=/tmp
o=gpurun_out/r04c6
mkdir -p $o
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
R3LIB=$PWD/manifold-based-optical-flow-method_amd/mofhip/libmofhip_r3.so
S=tools/gpu_step.sh
$S 600 $o/gputests.log python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread || exit 99
$S 400 $o/S1.json python3 bench.py --config S1 --steps 4 --warmup 1 --no-cpu-baseline --host-batches 0 || exit 99
$S 300 $o/S1s.json python3 bench.py --config S1s --steps 20 --warmup 2 --no-cpu-baseline --host-batches 0 || exit 99
run_pmc() {  # tag "counters" [MOFHIP_LIB]
  local tag=$1 ctr=$2 lib=$3
  mkdir -p $o/$tag
  MOFHIP_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $o/$tag -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/$tag/bench.json 2> $o/$tag/err.txt || exit 99
}
run_pmc sq_before "$SQ" $R3LIB
run_pmc sq_after "$SQ" ""
run_pmc fetch_before FETCH_SIZE $R3LIB
run_pmc fetch_after FETCH_SIZE ""
run_pmc write_before WRITE_SIZE $R3LIB
run_pmc write_after WRITE_SIZE ""
bash tools/profile_c3.sh r04 || exit 99
