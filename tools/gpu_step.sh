#!/bin/bash
# gpu_step.sh SECONDS LOG CMD... -- run one GPU step under its own time limit,
# output to LOG; exit status 0/1 (pass / ordinary failure) lets the caller
# continue, anything else (fault, abort, time limit) ends the call.
t=$1; log=$2; shift 2
timeout -k 10 "$t" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc $*" >> "$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_step] STOP rc=$rc: $*"; exit 99; fi
exit 0
