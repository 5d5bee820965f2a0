set -o pipefail
O=gpurun_out/r1s21; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_models_golden.py tests/test_gpu_pointsea.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo tests ok &&
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo bench ok &&
timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/bench_ps.json 2> $O/bench_ps.err && echo psbench ok
