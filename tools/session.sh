# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run: stem pool parity + PointSea trace.
set -o pipefail
O=gpurun_out/r5mp3; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pointsea.py tests/test_gpu_pointops.py -k "maxpool or pool or pointsea" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_run.sh $O trace_ps || exit 1
grep -i -E "pool" $O/trace_ps_kernel_stats_replay.csv | cut -c1-160
head -1 $O/trace_ps_window.txt
