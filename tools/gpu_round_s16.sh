set -o pipefail
O=gpurun_out/r1s16; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo tests ok &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && echo bench ok &&
timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/bench_ps.json 2> $O/bench_ps.err && echo psbench ok
