set -o pipefail
O=gpurun_out/r1s42; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo pytest ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing > $O/bench.json 2> $O/bench.err && echo bench ok &&
timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline --no-kernel-timing > $O/ps.json 2> $O/ps.err && echo ps ok
