set -o pipefail
O=gpurun_out/r1s5; mkdir -p $O
timeout -k 10 60 ./tools/fps_probe > $O/fps_probe.txt 2>&1 && echo probe ok &&
timeout -k 10 120 python tools/attn_bench.py 1 3 > $O/attn.txt 2>&1 && echo attn ok
