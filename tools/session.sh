# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5wh; mkdir -p $O; export TMPDIR=/tmp
for v in "PCOPS_WGRAD_BM=128 PCOPS_WGRAD_WGS=512" "PCOPS_WGRAD_BM=256 PCOPS_WGRAD_WGS=256" "PCOPS_WGRAD_BM=256 PCOPS_WGRAD_WGS=512" "PCOPS_WGRAD_BM=128 PCOPS_WGRAD_WGS=1024"; do
  echo "== $v" >> $O/ab.txt
  env $v PCOPS_WGRAD_MFMA=1 timeout -k 10 200 python tools/gemm_bench.py tuned 2>&1 | grep -o "^[0-9]*->[0-9]*\|product _wgrad [0-9]*us [0-9]*TF" | paste - - >> $O/ab.txt || exit 1
done
cat $O/ab.txt
