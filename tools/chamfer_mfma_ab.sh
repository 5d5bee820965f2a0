#!/bin/bash
# Chamfer screen A/B on the GPU box: tools/microbench.py per keep-test size of the MFMA screen, the
# Chamfer parity tests on the MFMA screen everywhere, then a same-box PCN bench A/B.
#   bash tools/chamfer_mfma_ab.sh <out-dir>
set -o pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
for cfg in "PCOPS_CHAMFER_MFMA=0" "PCOPS_CHAMFER_MFMA=2 PCOPS_CHAMFER_MFMA_SUB=32" \
           "PCOPS_CHAMFER_MFMA=2 PCOPS_CHAMFER_MFMA_SUB=64" "PCOPS_CHAMFER_MFMA=2 PCOPS_CHAMFER_MFMA_SUB=128"; do
  echo "== $cfg" >> "$OUT/chamfer_ab.txt"
  env $cfg timeout -k 10 120 python tools/microbench.py 2>&1 | grep -i chamfer >> "$OUT/chamfer_ab.txt" || exit 1
done
PCOPS_CHAMFER_MFMA=2 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k chamfer >> "$OUT/tests.txt" 2>&1 || exit 1
BENCH_AB="PCOPS_CHAMFER_MFMA=0;PCOPS_CHAMFER_MFMA=1;PCOPS_CHAMFER_MFMA=0;PCOPS_CHAMFER_MFMA=1" \
  bash tools/gpu_run.sh "$OUT" bench_ab
