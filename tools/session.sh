# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5sh; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pointsea.py -k "shared or counts" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -5 $O/pytest.log
bash tools/gpu_run.sh $O pmc_traffic
