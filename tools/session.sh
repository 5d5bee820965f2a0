# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5z; mkdir -p $O
export TMPDIR=/tmp
B="--model pointsea --no-cpu-baseline --no-fp32-leg --no-extra-legs"
for r in 1 2; do
  timeout -k 10 400 python bench.py $B > $O/ps_gtpf_$r.json 2>> $O/ps.err || exit 1
  timeout -k 10 400 python bench.py $B --no-gt-prefetch > $O/ps_nogtpf_$r.json 2>> $O/ps.err || exit 1
done
