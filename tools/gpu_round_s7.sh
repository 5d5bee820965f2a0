set -o pipefail
O=gpurun_out/r1s7; mkdir -p $O
PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 1000 python bench.py --tunableop tune --steps 3 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/tune_svd.json 2> $O/tune_svd.err; rc=$?; cp tuning/*.csv $O/ 2>/dev/null; echo "tune rc=$rc" && [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_svd_tuned.json 2> $O/bench_svd_tuned.err && echo bench ok
