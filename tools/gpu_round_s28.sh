set -o pipefail
O=gpurun_out/r1s28; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread -k "colsum or linear" > $O/t.log 2>&1 && echo tests ok &&
timeout -k 10 120 python tools/colsum_bench.py > $O/colsum.log 2>&1 && echo colsum ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo bench ok &&
timeout -k 10 200 python bench.py --model pointsea --no-cpu-baseline > $O/ps1.json 2> $O/ps1.err && echo ps1 ok
