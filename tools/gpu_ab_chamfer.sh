# Chamfer 16384^2 A/B: queries per lane (PCOPS_CHAMFER_Q) and the scalar
# round-1 kernel (tools/exp/ch_old), plus SQ counters of the default build.
set -o pipefail
O=${1:-gpurun_out/ab_chamfer}; mkdir -p $O; export TMPDIR=/tmp
for q in 1 2 4 8; do
  PCOPS_CHAMFER_Q=$q timeout -k 10 60 python tools/chamfer_bench.py 50 > $O/q$q.txt 2>&1 || exit 1
done
if [ -f tools/exp/ch_old/libpcops.so ]; then
  PCOPS_LIB_PATH=tools/exp/ch_old/libpcops.so timeout -k 10 60 python tools/chamfer_bench.py 50 > $O/old.txt 2>&1 || exit 1
fi
cat $O/q*.txt $O/old.txt 2>/dev/null | grep chamfer
