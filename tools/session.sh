# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5cm; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pointops.py tests/test_gpu_model.py tests/test_gpu_train_step.py tests/test_gpu_pointsea.py tests/test_gpu_sa_fused.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
export BENCH_AB="X=1;PCOPS_CHANNEL_MEAN=0;X=1;PCOPS_CHANNEL_MEAN=0"
bash tools/gpu_run.sh $O bench_ab || exit 1
grep -E '^==|ms_per_step' $O/bench_ab.txt | sed 's/.*"ms_per_step": \([0-9.]*\).*/\1/' | paste - -
