# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5rd; mkdir -p $O
export TMPDIR=/tmp
SH="16384x16384 2048x2048 512x2048 2048x512 256x256"
for rep in 1 2; do
for L in abl5/base/_lib/libpcops.so abl5/rd4/_lib/libpcops.so svdformer_pointsea_amd/_lib/libpcops.so abl5/rd16/_lib/libpcops.so; do
  for d in gauss surface; do
    PCOPS_LIB_PATH=$L CH_DATA=$d timeout -k 10 60 python tools/chamfer_bench.py 20 $SH >> $O/ab.txt 2>&1 || exit 1
  done
done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pointops.py -k "chamfer or Chamfer" > $O/pytest_chamfer.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_train_flat.py > $O/pytest_train.log 2>&1 || exit 1
tail -3 $O/pytest_chamfer.log $O/pytest_train.log
