# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_capture_fork.py tests/test_gpu_pointops.py tests/test_gpu_pointsea.py tests/test_gpu_model.py tests/test_gpu_sa_fused.py -x -v --timeout 300 --timeout-method thread -k "capture or fps or seprate or pointsea or replays or model or sa or chamfer" > $O/tests.log 2>&1 || exit 1
for d in gauss surface; do
  for L in abl5/base/_lib/libpcops.so svdformer_pointsea_amd/_lib/libpcops.so abl5/wpe6/_lib/libpcops.so; do
    PCOPS_LIB_PATH=$PWD/$L CH_DATA=$d timeout -k 10 120 python tools/chamfer_bench.py 20 16384x16384 2048x16384 >> $O/ch.txt 2>&1 || exit 1
  done
done
for f in 1 0 1 0; do
  PCOPS_FPS_SHARE=$f timeout -k 10 400 python bench.py --no-cpu-baseline --no-fp32-leg --no-extra-legs > $O/pcn_share$f.json.$RANDOM 2>> $O/pcn_share$f.err || exit 1
done
for f in 1 0; do
  PCOPS_FPS_SHARE=$f timeout -k 10 400 python bench.py --model pointsea --no-cpu-baseline --no-fp32-leg --no-extra-legs > $O/ps_share$f.json 2>> $O/ps_share$f.err || exit 1
done
