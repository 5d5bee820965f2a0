# Is the split-K weight gradient (bmm partials + pcops_sum_rows, attention._wgrad) still worth its
# launches once TunableOp has tuned the plain long-K GEMMs too?  1) tune with the split off (the
# plain g^T x shapes join the committed table), 2) same-box A/B of the PCN step, split on / off.
set -o pipefail
OUT=gpurun_out/r6j
mkdir -p $OUT
cp tuning/tunableop_svdformer_gfx950.csv $OUT/before.csv
PCOPS_WGRAD_SPLITK=0 timeout -k 10 600 python bench.py --tunableop tune --steps 3 --warmup 2 --no-cpu-baseline \
  --no-fp32-leg --no-extra-legs --no-kernel-timing > $OUT/tune.json 2> $OUT/tune.err || exit 1
cp tuning/tunableop_svdformer_gfx950.csv $OUT/after.csv
wc -l $OUT/before.csv $OUT/after.csv
for g in 1 0 1 0; do
  echo "== PCOPS_WGRAD_SPLITK=$g" >> $OUT/ab.txt
  PCOPS_WGRAD_SPLITK=$g timeout -k 10 400 python bench.py --no-cpu-baseline --no-fp32-leg --no-extra-legs \
    --no-kernel-timing --steps 20 --warmup 3 >> $OUT/ab.txt 2>> $OUT/ab.err || exit 1
done
