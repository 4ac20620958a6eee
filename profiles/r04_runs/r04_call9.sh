#!/bin/bash
# round-4 call 9: why k_residual_x3sm is slow -- per-kernel times by batch
# (locality of the interleaved operands), XCD mapping by system group
# (MOF_RES_SM_MAP=1), natural row order (MOF_RES_SM_NAT=1); FETCH_SIZE of
# the variants
export TMPDIR=/tmp
o=gpurun_out/r04c9
mkdir -p $o
prof() {  # tag batch env...
  local tag=$1 bt=$2; shift 2
  mkdir -p $o/$tag
  env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$tag -o run -- \
      python3 bench.py --steps 2 --warmup 1 --batch $bt --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/$tag/bench.json 2> $o/$tag/err.txt || exit 99
}
prof rcn_b64 64 MOF_RES_SM=0
prof sm_b64 64 MOF_RES_SM=1
prof sm_b512_map1 512 MOF_RES_SM=1 MOF_RES_SM_MAP=1
prof sm_b512_nat 512 MOF_RES_SM=1 MOF_RES_SM_NAT=1
prof sm_b512_map1_nat 512 MOF_RES_SM=1 MOF_RES_SM_MAP=1 MOF_RES_SM_NAT=1
pmc() {  # tag counters env...
  local tag=$1 ctr=$2; shift 2
  mkdir -p $o/$tag
  env "$@" timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $o/$tag -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 \
      > $o/$tag/bench.json 2> $o/$tag/err.txt || exit 99
}
pmc fetch_sm FETCH_SIZE MOF_RES_SM=1
pmc fetch_sm_map1_nat FETCH_SIZE MOF_RES_SM=1 MOF_RES_SM_MAP=1 MOF_RES_SM_NAT=1
pmc hit_sm "TCC_HIT_sum TCC_MISS_sum" MOF_RES_SM=1
