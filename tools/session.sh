# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r4rule; mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --no-fp32-leg --no-extra-legs"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/pcn_pairs_$i.json 2> $O/pcn_pairs_$i.err || exit 1
  PCOPS_CHAMFER_CULL_PAIRS=0 timeout -k 10 300 python bench.py $B > $O/pcn_all_$i.json 2> $O/pcn_all_$i.err || exit 1
done
PCOPS_CHAMFER_CULL_PAIRS=0 bash tools/gpu_run.sh $O/all tests || exit 1
