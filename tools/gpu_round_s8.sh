set -o pipefail
O=gpurun_out/r1s8; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pointops.py tests/test_models_golden.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo tests ok &&
timeout -k 10 120 python tools/knn_bench.py > $O/knn_v2.txt 2>&1 && PCOPS_KNN_V1=1 timeout -k 10 120 python tools/knn_bench.py > $O/knn_v1.txt 2>&1 && echo knn ok &&
PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 1000 python bench.py --model pointsea --tunableop tune --steps 3 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/tune_ps.json 2> $O/tune_ps.err; rc=$?; cp tuning/tunableop_pointsea*.csv $O/ 2>/dev/null; echo "tune rc=$rc" && [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/bench_ps.json 2> $O/bench_ps.err && echo psbench ok
