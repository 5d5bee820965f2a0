set -o pipefail
O=gpurun_out/r1s10; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pointops.py tests/test_gpu_pointsea.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && echo tests ok &&
timeout -k 10 60 ./tools/fps_probe > $O/fps_probe.txt 2>&1 && echo probe ok &&
timeout -k 10 120 python tools/microbench.py > $O/micro_v2.txt 2>&1 && PCOPS_FPS_V1=1 timeout -k 10 120 python tools/microbench.py > $O/micro_v1.txt 2>&1 && echo micro ok
