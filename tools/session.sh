# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
bash tools/gpu_run.sh gpurun_out/r5f2 tests smoke bench trace
