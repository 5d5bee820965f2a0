set -o pipefail
O=gpurun_out/r1s39; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread -k "layernorm" > $O/t.log 2>&1 && echo tests ok &&
timeout -k 10 300 env PCOPS_LN_CH2=1 python bench.py --no-cpu-baseline > $O/ch2.json 2> $O/ch2.err && echo ch2 ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/ch1.json 2> $O/ch1.err && echo ch1 ok
