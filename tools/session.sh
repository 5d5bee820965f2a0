set -o pipefail
O=gpurun_out/r4d1; mkdir -p $O
export TMPDIR=/tmp
export PYTEST_K="flat_adam or dist"
bash tools/gpu_run.sh $O tests_k dist1
