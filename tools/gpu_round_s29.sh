set -o pipefail
O=gpurun_out/r1s29; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread -k "colsum or linear or layernorm" > $O/t.log 2>&1 && echo tests ok &&
timeout -k 10 100 python tools/colsum_bench.py > $O/colsum.log 2>&1 &&
PCOPS_COLSUM_BLOCKS=1024 PCOPS_COLSUM_CHUNKS=256 timeout -k 10 100 python tools/colsum_bench.py pcops >> $O/colsum.log 2>&1 &&
PCOPS_COLSUM_BLOCKS=1024 PCOPS_COLSUM_CHUNKS=1024 timeout -k 10 100 python tools/colsum_bench.py pcops >> $O/colsum.log 2>&1 &&
PCOPS_COLSUM_BLOCKS=4096 PCOPS_COLSUM_CHUNKS=1024 timeout -k 10 100 python tools/colsum_bench.py pcops >> $O/colsum.log 2>&1 &&
PCOPS_COLSUM_BLOCKS=512 PCOPS_COLSUM_CHUNKS=256 timeout -k 10 100 python tools/colsum_bench.py pcops >> $O/colsum.log 2>&1 && echo colsum ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo bench ok
