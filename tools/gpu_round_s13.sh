set -o pipefail
O=gpurun_out/r1s13; mkdir -p $O
timeout -k 10 60 ./tools/fps_probe > $O/probe_split8.txt 2>&1 && PCOPS_FPS_SPLIT_PPT=16 timeout -k 10 60 ./tools/fps_probe > $O/probe_split16.txt 2>&1 && echo probe ok &&
PCOPS_FPS_SPLIT_PPT=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_pointops.py -x -q -k "fps or furthest" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo tests ok
