set -o pipefail
O=gpurun_out/r4w; mkdir -p $O
export TMPDIR=/tmp
export PYTEST_K="glue_fusions"
bash tools/gpu_run.sh $O tests_k || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/ps_new_$i.json 2> $O/ps_new_$i.err || exit 1
  PCOPS_PS_CAT16=0 timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/ps_nocat_$i.json 2> $O/ps_nocat_$i.err || exit 1
done
