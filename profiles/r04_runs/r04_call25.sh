#!/bin/bash
# round-4 call 25: SQ issue / wait counters of the final build at the default
# batch (1024), one pass
export TMPDIR=/tmp
bash tools/pmc_issue.sh r04b_b1024 --parity-samples 0 --host-batches 0 || exit 99
