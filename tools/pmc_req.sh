#!/bin/bash
# pmc_req.sh TAG [VARIANT] -- one rocprofv3 pass of the L2 -> fabric read
# request counters by size (TCC_EA0_RDREQ total, 32 B, 64 B, 128 B: 4 TCC
# counters, the limit of one pass) of a short bench.py run, per dispatch,
# under gpurun_out/pmcr_TAG/. Bytes = 32 n32 + 64 n64 + 128 n128 calibrate
# FETCH_SIZE for gather-shaped kernels (MI355X_MICROARCH.md §HBM: the x2
# correction holds for wide streaming reads only). VARIANT: a
# mofhip/libmofhip_VARIANT.so (tools/build_variant.sh) instead of the default.
tag=$1; v=${2:-base}
lib=""
[ "$v" != base ] && lib=$PWD/manifold-based-optical-flow-method_amd/mofhip/libmofhip_$v.so
out=gpurun_out/pmcr_$tag/$v
mkdir -p $out
export TMPDIR=/tmp
MOFHIP_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum \
    TCC_EA0_RDREQ_128B_sum --output-format csv -d $out -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 > $out/bench.json 2> $out/err.txt || exit 99
