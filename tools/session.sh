# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_capture_fork.py -x -v --timeout 300 --timeout-method thread > $O/cap_tests.log 2>&1 || exit 1
B="--model pointsea --no-cpu-baseline --no-fp32-leg --no-extra-legs"
for f in 1 0 1 0; do
  PCOPS_LOCAL_FPS_FORK=$f timeout -k 10 400 python bench.py $B > $O/ps_fork$f.json.$RANDOM 2>> $O/ps_fork$f.err || exit 1
done
