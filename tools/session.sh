# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r4ch8; mkdir -p $O
export TMPDIR=/tmp
export PYTEST_K="culled or nonfinite_scan or chamfer"
bash tools/gpu_run.sh $O tests_k || exit 1
PCOPS_CHAMFER_CULL_ES=0 PYTEST_K="culled" bash tools/gpu_run.sh $O/es0 tests_k || exit 1
for d in gauss surface; do
  for es in 1 0; do
    PCOPS_CHAMFER_CULL_ES=$es CH_DATA=$d timeout -k 10 120 python tools/chamfer_bench.py 20 16384x16384 8192x8192 >> $O/ch_es$es.txt 2>&1 || exit 1
  done
done
B="--no-cpu-baseline --no-fp32-leg --no-extra-legs"
for i in 1 2; do
  PCOPS_CHAMFER_CULL_ES=0 timeout -k 10 300 python bench.py $B > $O/pcn_es0_$i.json 2> $O/pcn_es0_$i.err || exit 1
  timeout -k 10 300 python bench.py $B > $O/pcn_es1_$i.json 2> $O/pcn_es1_$i.err || exit 1
done
for i in 1; do
  PCOPS_CHAMFER_MFMA=1 timeout -k 10 300 python bench.py $B > $O/pcn_mfma1_$i.json 2> $O/pcn_mfma1_$i.err || exit 1
done
