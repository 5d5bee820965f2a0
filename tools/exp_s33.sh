set -o pipefail
mkdir -p gpurun_out/s34
for cfg in "PCOPS_CHAMFER_MFMA=0" "PCOPS_CHAMFER_MFMA=2 PCOPS_CHAMFER_MFMA_SUB=32" "PCOPS_CHAMFER_MFMA=2 PCOPS_CHAMFER_MFMA_SUB=64"; do
  echo "== $cfg" >> gpurun_out/s34/chamfer_ab.txt
  env $cfg timeout -k 10 120 python tools/microbench.py 2>&1 | grep -i chamfer >> gpurun_out/s34/chamfer_ab.txt || exit 1
done
PCOPS_CHAMFER_MFMA=2 PCOPS_CHAMFER_MFMA_SUB=32 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k chamfer >> gpurun_out/s34/tests.txt 2>&1 || exit 1
BENCH_AB="PCOPS_CHAMFER_MFMA=1;PCOPS_CHAMFER_MFMA=2 PCOPS_CHAMFER_MFMA_SUB=64;PCOPS_CHAMFER_MFMA=1;PCOPS_CHAMFER_MFMA=2 PCOPS_CHAMFER_MFMA_SUB=64" bash tools/gpu_run.sh gpurun_out/s34 bench_ab
