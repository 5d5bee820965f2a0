# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r4xcd; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/ablc/base/libpcops.so
PYTEST_K="culled or nonfinite_scan" bash tools/gpu_run.sh $O tests_k || exit 1
for d in gauss surface; do
  CH_DATA=$d timeout -k 10 120 python tools/chamfer_bench.py 20 16384x16384 >> $O/ch_xcd.txt 2>&1 || exit 1
  PCOPS_LIB_PATH=$L CH_DATA=$d timeout -k 10 120 python tools/chamfer_bench.py 20 16384x16384 >> $O/ch_base.txt 2>&1 || exit 1
done
B="--no-cpu-baseline --no-fp32-leg --no-extra-legs"
for i in 1 2; do
  PCOPS_LIB_PATH=$L timeout -k 10 300 python bench.py $B > $O/pcn_base_$i.json 2> $O/pcn_base_$i.err || exit 1
  timeout -k 10 300 python bench.py $B > $O/pcn_xcd_$i.json 2> $O/pcn_xcd_$i.err || exit 1
done
bash tools/gpu_run.sh $O tests smoke || exit 1
