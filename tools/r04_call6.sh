#!/bin/bash
# round-4 call 6: counters of the setup kernels before (the round-3 library,
# libmofhip_r3.so) and after (this build): SQ issue / wait shares, FETCH_SIZE,
# WRITE_SIZE, each pass its own run; then the final profile of the default
# line (kernel trace + stats, separate FETCH / WRITE passes)
export TMPDIR=/tmp
o=gpurun_out/r04c6
mkdir -p $o
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
R3LIB=$PWD/manifold-based-optical-flow-method_amd/mofhip/libmofhip_r3.so
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
