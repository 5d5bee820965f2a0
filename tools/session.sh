set -o pipefail
O=gpurun_out/r4s; mkdir -p $O
export TMPDIR=/tmp
export PYTEST_K="knn or gelu or edgeconv or group_local or sa_group"
bash tools/gpu_run.sh $O tests_k || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/knn_bench.py \
  > $O/knn.txt 2>&1 || exit 1
f=$(find $O/prof -name '*kernel_stats.csv' -print -quit); cp "$f" $O/knn_stats.csv; find $O/prof -name '*kernel_trace.csv' -delete
B="--no-cpu-baseline --no-fp32-leg --no-extra-legs"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/pcn_gelu_$i.json 2> $O/pcn_gelu_$i.err || exit 1
  PCOPS_GELU_FWD=0 timeout -k 10 300 python bench.py $B > $O/pcn_torchgelu_$i.json 2> $O/pcn_torchgelu_$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/ps_$i.json 2> $O/ps_$i.err || exit 1
done
