# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r4pmc; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_run.sh $O pmc_traffic || exit 1
