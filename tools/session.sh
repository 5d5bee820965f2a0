# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5ns; mkdir -p $O; export TMPDIR=/tmp
NEW=PCOPS_LIB_PATH=abl6/noslp/libpcops.so
env $NEW timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_attention.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
export ATTN_AB="$NEW;X=old;$NEW;X=old" ATTN_SHAPES="0 1 3"
bash tools/gpu_run.sh $O attn_ab || exit 1
grep -E "^==|bwd|dkv" $O/attn_ab.txt | head -60
export BENCH_AB="$NEW;X=old;$NEW;X=old"
bash tools/gpu_run.sh $O bench_ab || exit 1
grep -E '^==|ms_per_step' $O/bench_ab.txt | sed 's/.*"ms_per_step": \([0-9.]*\).*/\1/' | paste - -
