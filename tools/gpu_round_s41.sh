set -o pipefail
O=gpurun_out/r1s41; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread -k "bf16 or golden or forward" > $O/t.log 2>&1 && echo tests ok &&
timeout -k 10 200 env PCOPS_LIB_PATH=svdformer_pointsea_amd/_lib/libpcops_defer0.so python tools/attn_bench.py > $O/attn.log 2>&1 &&
timeout -k 10 200 python tools/attn_bench.py >> $O/attn.log 2>&1 && echo attn ok &&
timeout -k 10 300 env PCOPS_LIB_PATH=svdformer_pointsea_amd/_lib/libpcops_defer0.so python bench.py --no-cpu-baseline --no-kernel-timing > $O/d0.json 2> $O/d0.err && echo d0 ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing > $O/d8.json 2> $O/d8.err && echo d8 ok
