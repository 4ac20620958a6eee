#!/bin/bash
# pmc_issue.sh TAG [bench args...] -- one rocprofv3 SQ-counter pass of a short
# bench.py run (issue / wait / VALU counters per dispatch), under
# gpurun_out/pmcq_TAG/ (MI355X_MICROARCH.md: <= 8 SQ counters per pass,
# counters in their own pass, no trace domains beside --pmc).
tag=$1; shift
out=gpurun_out/pmcq_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $out -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $out/bench.json 2> $out/err.txt || exit 99
