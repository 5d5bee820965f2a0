# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run: the final tree's GPU tests and smoke.
set -o pipefail
O=gpurun_out/r5end; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_run.sh $O tests smoke || exit 1
tail -1 $O/pytest_gpu.log; tail -1 $O/smoke.log
