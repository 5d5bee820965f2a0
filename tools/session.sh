set -o pipefail
O=gpurun_out/r4m; mkdir -p $O
export PYTEST_K="knn or group_local or edgeconv or add_posemb"
bash tools/gpu_run.sh $O tests_k || exit 1
for i in 1 2; do
  timeout -k 10 120 python tools/knn_bench.py > $O/knn_c3_$i.txt 2>&1 || exit 1
  PCOPS_KNN_C3=0 timeout -k 10 120 python tools/knn_bench.py > $O/knn_c2_$i.txt 2>&1 || exit 1
done
bash tools/gpu_run.sh $O bench_ps
