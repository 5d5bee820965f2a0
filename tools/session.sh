# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r4min; mkdir -p $O
export TMPDIR=/tmp
PCOPS_CHAMFER_CULL_MIN=256 PYTEST_K="culled" bash tools/gpu_run.sh $O/t tests_k || exit 1
for n in 512x512 2048x2048 2048x16384; do
  for m in 4096 256; do
    PCOPS_CHAMFER_CULL_MIN=$m CH_DATA=surface timeout -k 10 120 python tools/chamfer_bench.py 20 $n >> $O/ch_min$m.txt 2>&1 || exit 1
  done
done
B="--no-cpu-baseline --no-fp32-leg --no-extra-legs"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/pcn_4096_$i.json 2> $O/pcn_4096_$i.err || exit 1
  PCOPS_CHAMFER_CULL_MIN=256 timeout -k 10 300 python bench.py $B > $O/pcn_256_$i.json 2> $O/pcn_256_$i.err || exit 1
done
