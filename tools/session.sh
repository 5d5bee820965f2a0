# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5bnp; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batchnorm.py tests/test_gpu_model.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/bn_bench.py > $O/bn_bench.txt 2>&1 || exit 1
cat $O/bn_bench.txt
OLD=PCOPS_LIB_PATH=abl6/libpcops_old.so
export BENCH_AB="X=new;$OLD;X=new;$OLD"
bash tools/gpu_run.sh $O bench_ab || exit 1
grep -E '^==|ms_per_step' $O/bench_ab.txt | sed 's/.*"ms_per_step": \([0-9.]*\).*/\1/' | paste - -
