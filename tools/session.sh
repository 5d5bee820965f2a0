# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5ov3; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pointops.py -k "chamfer or Chamfer" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
SH="512x2048 2048x2048 256x256"
for L in abl6/base/_lib/libpcops.so svdformer_pointsea_amd/_lib/libpcops.so; do
  for d in same gauss; do
    PCOPS_LIB_PATH=$L CH_DATA=$d timeout -k 10 60 python tools/chamfer_bench.py 20 $SH >> $O/ab.txt 2>&1 || exit 1
  done
done
grep chamfer $O/ab.txt
export BENCH_AB="PCOPS_LIB_PATH=abl6/base/_lib/libpcops.so;X=1;PCOPS_LIB_PATH=abl6/base/_lib/libpcops.so;X=1"
bash tools/gpu_run.sh $O bench_ab || exit 1
grep -E '^==|ms_per_step' $O/bench_ab.txt | sed 's/.*"ms_per_step": \([0-9.]*\).*/\1/' | paste - -
