#!/bin/bash
# Round 6: boundary sweeps on the ring's own SELL matrix (bits vs the
# round-5 kernel; iterations and rates with the sweeps on every open patch
# and coarse smoothing)
set -o pipefail
o=gpurun_out/r06bsw2; mkdir -p $o
L=$PWD/manifold-based-optical-flow-method_amd/mofhip
step() { local n=$1; shift; timeout -k 10 ${T:-240} "$@" > $o/$n.out 2> $o/$n.err; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="--steps 3 --warmup 1 --no-cpu-baseline --parity-samples 2 --host-batches 0 --legs none"
step vh_s1s_new python3 tools/vhash.py S1s 97
MOFHIP_LIB=$L/libmofhip_old.so step vh_s1s_old python3 tools/vhash.py S1s 97
MOF_AMG_BSW=2 step vh_s1m_new python3 tools/vhash.py S1m 13
MOF_AMG_BSW=2 MOFHIP_LIB=$L/libmofhip_old.so step vh_s1m_old python3 tools/vhash.py S1m 13
MOF_AMG_BSW=1 step vh1_s1m_new python3 tools/vhash.py S1m 13
MOF_AMG_BSW=1 MOFHIP_LIB=$L/libmofhip_old.so step vh1_s1m_old python3 tools/vhash.py S1m 13
cat $o/vh*.out
step t_bsw python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_amg.py -k boundary_sweeps
step s1s_new python3 bench.py --config S1s --steps 20 --warmup 2 --no-cpu-baseline --parity-samples 2 --host-batches 0 --legs none
MOFHIP_LIB=$L/libmofhip_old.so step s1s_old python3 bench.py --config S1s --steps 20 --warmup 2 --no-cpu-baseline --parity-samples 2 --host-batches 0 --legs none
step s1m_base python3 bench.py --config S1m $B
MOF_AMG_BSW=2 step s1m_bsw python3 bench.py --config S1m $B
MOF_AMG_BSW=2 MOFHIP_LIB=$L/libmofhip_sm2.so step s1m_bsw_sm2 python3 bench.py --config S1m $B
step s1_base python3 bench.py --config S1 $B
MOF_AMG_BSW=2 step s1_bsw python3 bench.py --config S1 $B
MOF_AMG_BSW=2 MOFHIP_LIB=$L/libmofhip_sm2.so step s1_bsw_sm2 python3 bench.py --config S1 $B
MOF_AMG_BSW=3 MOFHIP_LIB=$L/libmofhip_sm2.so step s1_bsw3_sm2 python3 bench.py --config S1 $B
MOF_AMG_BSW=1 MOFHIP_LIB=$L/libmofhip_sm2.so step s1_bsw1_sm2 python3 bench.py --config S1 $B
for f in $o/s1*.out; do python3 -c "import json,sys;l=json.loads(open(sys.argv[1]).readline());print(sys.argv[1].split('/')[-1],l['value'],l['solver']['pcg_iterations_per_timestep'],l['solver'].get('recovered'),(l.get('parity') or {}).get('max_abs_err'))" $f; done
MOF_AMG_BSW=2 MOFHIP_LIB=$L/libmofhip_sm2.so step prof_s1_bsw_sm2 rocprofv3 --kernel-trace --stats -d $o/prof_s1_bsw_sm2 -o run -- python3 bench.py --config S1 --steps 2 --warmup 1 --no-cpu-baseline --parity-samples 0 --host-batches 0 --legs none
