# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5x; mkdir -p $O
export TMPDIR=/tmp
for d in gauss surface; do
  for L in svdformer_pointsea_amd/_lib/libpcops.so abl5/u4/_lib/libpcops.so abl5/u8/_lib/libpcops.so svdformer_pointsea_amd/_lib/libpcops.so; do
    PCOPS_LIB_PATH=$PWD/$L CH_DATA=$d timeout -k 10 120 python tools/chamfer_bench.py 20 16384x16384 2048x16384 >> $O/ch_unroll.txt 2>&1 || exit 1
  done
  for r in 1 2; do
    CH_DATA=$d timeout -k 10 120 python tools/chamfer_bench.py 30 2048x2048 512x2048 2048x512 256x256 1024x2048 >> $O/ch_small.txt 2>&1 || exit 1
    PCOPS_CHAMFER_CULL_PAIRS=0 PCOPS_CHAMFER_CULL_MIN=1 CH_DATA=$d timeout -k 10 120 python tools/chamfer_bench.py 30 2048x2048 512x2048 2048x512 256x256 1024x2048 | sed 's/^/FORCED /' >> $O/ch_small.txt 2>&1 || exit 1
  done
done
