set -o pipefail
O=gpurun_out/r1s38; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_pointops.py -x -q --timeout 120 --timeout-method thread -k pcsa > $O/t.log 2>&1 && echo tests ok &&
timeout -k 10 120 python tools/pcsa_bench.py > $O/pcsa.log 2>&1 &&
timeout -k 10 120 env PCOPS_PCSA_V1=1 python tools/pcsa_bench.py >> $O/pcsa.log 2>&1 && echo pcsa ok &&
timeout -k 10 300 env PCOPS_PCSA_V1=1 python bench.py --no-cpu-baseline --no-kernel-timing > $O/v1.json 2> $O/v1.err && echo v1 ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing > $O/wave.json 2> $O/wave.err && echo wave ok
