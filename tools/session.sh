# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5bn2; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
for v in 0 1; do
  echo "== $v" >> $O/ps.txt
  PCOPS_BN_FUSED_FINAL=$v timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline --no-fp32-leg --no-extra-legs --no-kernel-timing --steps 20 --warmup 3 >> $O/ps.txt 2>> $O/ps.err || exit 1
done
done
grep -E '^==|ms_per_step' $O/ps.txt | sed 's/.*"ms_per_step": \([0-9.]*\).*/\1/' | paste - -
