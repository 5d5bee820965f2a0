set -o pipefail
O=gpurun_out/r1s3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pointsea.py -x -v --timeout 120 --timeout-method thread > $O/pytest_pointsea.log 2>&1 && echo pstests ok &&
timeout -k 10 400 python bench.py --model pointsea > $O/bench_pointsea.json 2> $O/bench_pointsea.err && echo psbench ok &&
timeout -k 10 300 python tools/step_profile.py --model svdformer > $O/step_svd.txt 2>&1 && echo prof1 ok &&
timeout -k 10 300 python tools/step_profile.py --model pointsea > $O/step_ps.txt 2>&1 && echo prof2 ok
