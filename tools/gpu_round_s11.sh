set -o pipefail
O=gpurun_out/r1s11; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_pointops.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo tests ok &&
timeout -k 10 120 python tools/attn_bench.py 0 1 2 3 4 > $O/attn.txt 2>&1 && echo attn ok &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && echo bench ok
