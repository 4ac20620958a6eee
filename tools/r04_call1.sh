#!/bin/bash
# round-4 call 1: two batches in flight (tools/streams2.py) and the coarse
# Galerkin product by gather entry (libmofhip_gal3.so) against the default build
mkdir -p gpurun_out/r04c1
S=tools/gpu_step.sh
$S 400 gpurun_out/r04c1/streams_512.jsonl python3 -u tools/streams2.py C3 512 6 || exit 99
$S 400 gpurun_out/r04c1/streams_256.jsonl python3 -u tools/streams2.py C3 256 12 || exit 99
AB_REPS=2 bash tools/ab_bench.sh r04gal3 gal3 || exit 99
