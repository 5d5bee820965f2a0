set -o pipefail
O=gpurun_out/r4y; mkdir -p $O
export TMPDIR=/tmp
export PYTEST_K="flat_adam or train_step or checkpoint"
bash tools/gpu_run.sh $O tests_k || exit 1
B="--no-cpu-baseline --no-fp32-leg --no-extra-legs"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/pcn_flat_$i.json 2> $O/pcn_flat_$i.err || exit 1
  PCOPS_FLAT_ADAM=0 timeout -k 10 300 python bench.py $B > $O/pcn_torch_$i.json 2> $O/pcn_torch_$i.err || exit 1
done
timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/ps_flat.json 2> $O/ps_flat.err || exit 1
PCOPS_FLAT_ADAM=0 timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/ps_torch.json 2> $O/ps_torch.err || exit 1
