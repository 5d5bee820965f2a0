# Chamfer A/B at the step's shapes: queries per lane (PCOPS_CHAMFER_Q) x
# screened / direct kernel (PCOPS_CHAMFER_SCREEN).
set -o pipefail
O=${1:-gpurun_out/ab_chamfer}; mkdir -p $O; export TMPDIR=/tmp
SH="16384x16384 2048x2048 512x2048 2048x512 256x256"
timeout -k 10 60 python tools/chamfer_bench.py 20 $SH > $O/auto.txt 2>&1 || exit 1
for q in 1 2 4; do
  for sc in 0 1; do
    PCOPS_CHAMFER_Q=$q PCOPS_CHAMFER_SCREEN=$sc timeout -k 10 60 python tools/chamfer_bench.py 20 $SH \
      > $O/q${q}_s${sc}.txt 2>&1 || exit 1
  done
done
cat $O/*.txt | grep chamfer
