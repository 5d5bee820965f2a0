set -o pipefail
O=gpurun_out/r1s18; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pointops.py tests/test_models_golden.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo tests ok &&
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo bench ok &&
timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/r1s18/gemm.txt 2>&1 && timeout -k 10 120 python tools/gemm_bench.py tuned > gpurun_out/r1s18/gemm_tuned.txt 2>&1 && echo gemm ok
