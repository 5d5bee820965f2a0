# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r4ch7; mkdir -p $O
export TMPDIR=/tmp
export PYTEST_K="culled or nonfinite_scan or chamfer_screen"
bash tools/gpu_run.sh $O tests_k || exit 1
for d in gauss surface; do
  CH_DATA=$d timeout -k 10 120 python tools/chamfer_bench.py 20 16384x16384 8192x8192 >> $O/ch.txt 2>&1 || exit 1
done
B="--no-cpu-baseline --no-fp32-leg --no-extra-legs"
for i in 1 2; do
  PCOPS_CHAMFER_CULL=0 timeout -k 10 300 python bench.py $B > $O/pcn_screen_$i.json 2> $O/pcn_screen_$i.err || exit 1
  timeout -k 10 300 python bench.py $B > $O/pcn_cull_$i.json 2> $O/pcn_cull_$i.err || exit 1
done
