set -o pipefail
mkdir -p gpurun_out/bsw
for cfg in S1s S1; do
  for v in 0 2 0 2; do
    MOF_AMG_BSW=$v timeout -k 10 240 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/bsw/${cfg}_bsw${v}_$RANDOM.json 2> gpurun_out/bsw/err_${cfg}_$v.log || exit 1
  done
done
