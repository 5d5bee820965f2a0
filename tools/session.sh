# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r4ps; mkdir -p $O
export TMPDIR=/tmp
P="--model pointsea --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 300 python bench.py $P > $O/ps_default_$i.json 2> $O/ps_default_$i.err || exit 1
  PCOPS_CHAMFER_CULL=0 timeout -k 10 300 python bench.py $P > $O/ps_cull0_$i.json 2> $O/ps_cull0_$i.err || exit 1
  PCOPS_CHAMFER_MFMA=1 timeout -k 10 300 python bench.py $P > $O/ps_mfma1_$i.json 2> $O/ps_mfma1_$i.err || exit 1
done
