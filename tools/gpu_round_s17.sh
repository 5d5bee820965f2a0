set -o pipefail
O=gpurun_out/r1s17; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread > $O/pytest_attn.log 2>&1 && echo tests ok &&
timeout -k 10 120 python tools/attn_bench.py 1 3 > $O/attn_split.txt 2>&1 && PCOPS_DKV_SPLIT=0 timeout -k 10 120 python tools/attn_bench.py 1 3 > $O/attn_nosplit.txt 2>&1 && echo attn ok &&
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo bench ok
