set -o pipefail
O=gpurun_out/r1s15; mkdir -p $O
PCOPS_FPS_SPLIT_PPT=32 timeout -k 10 60 ./tools/fps_probe > $O/probe_split32.txt 2>&1 && echo probe ok &&
PCOPS_FPS_SPLIT_PPT=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_pointops.py -x -q -k "fps or furthest" --timeout 120 --timeout-method thread > $O/pytest32.log 2>&1 && echo tests32 ok
