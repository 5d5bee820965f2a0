set -o pipefail
O=gpurun_out/r4t2; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_run.sh $O trace pmc_traffic
