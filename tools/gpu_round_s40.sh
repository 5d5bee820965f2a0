set -o pipefail
O=gpurun_out/r1s40; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 && echo tests ok &&
timeout -k 10 300 env PCOPS_BLOCKSUM16=0 python bench.py --no-cpu-baseline --no-kernel-timing > $O/off.json 2> $O/off.err && echo off ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing > $O/on.json 2> $O/on.err && echo on ok
