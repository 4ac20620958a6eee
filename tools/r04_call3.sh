#!/bin/bash
# round-4 call 3: counters of the setup kernels before / after (SQ issue and
# wait shares, FETCH / WRITE bytes): "before" = the round-3 kernels
# (MOF_RESIDUAL=rcn, MOF_GAL3_ENT=0, MOF_ASM_G3=0), "after" = this build's
# defaults; then the final profile of the default line (kernel trace + stats,
# separate FETCH_SIZE / WRITE_SIZE passes)
export TMPDIR=/tmp
o=gpurun_out/r04c3
mkdir -p $o
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
run_pmc() {  # tag counters env...
  local tag=$1 ctr=$2; shift 2
  mkdir -p $o/$tag
  env "$@" timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $o/$tag -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/$tag/bench.json 2> $o/$tag/err.txt || exit 99
}
run_pmc sq_before "$SQ" MOF_RESIDUAL=rcn MOF_GAL3_ENT=0 MOF_ASM_G3=0
run_pmc sq_after "$SQ" MOF_PCG_STALL=64
run_pmc fetch_before FETCH_SIZE MOF_RESIDUAL=rcn MOF_GAL3_ENT=0 MOF_ASM_G3=0
run_pmc fetch_after FETCH_SIZE MOF_PCG_STALL=64
run_pmc write_before WRITE_SIZE MOF_RESIDUAL=rcn MOF_GAL3_ENT=0 MOF_ASM_G3=0
run_pmc write_after WRITE_SIZE MOF_PCG_STALL=64
bash tools/profile_c3.sh r04 || exit 99
