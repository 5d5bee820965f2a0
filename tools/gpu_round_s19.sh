set -o pipefail
O=gpurun_out/r1s19; mkdir -p $O
timeout -k 10 200 python tools/gemm_bench.py > $O/gemm.txt 2>&1 && echo gemm ok
