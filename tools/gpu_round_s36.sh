set -o pipefail
O=gpurun_out/r1s36; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_pointsea.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 && echo tests ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo bench ok &&
timeout -k 10 200 python bench.py --model pointsea --no-cpu-baseline > $O/ps1.json 2> $O/ps1.err && echo ps1 ok
