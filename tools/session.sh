set -o pipefail
O=gpurun_out/r4v; mkdir -p $O
export TMPDIR=/tmp
export PYTEST_K="blend or pair_input or pointsea or models_golden"
bash tools/gpu_run.sh $O tests_k || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/ps_new_$i.json 2> $O/ps_new_$i.err || exit 1
  PCOPS_BLEND=0 timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/ps_noblend_$i.json 2> $O/ps_noblend_$i.err || exit 1
done
