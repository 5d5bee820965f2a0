set -o pipefail
O=gpurun_out/r4pm; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_run.sh $O pmc_attn trace_ps
