set -o pipefail
O=gpurun_out/r4z; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_run.sh $O tests smoke bench
