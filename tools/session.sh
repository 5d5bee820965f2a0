# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5mw3; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pointops.py tests/test_gpu_pointsea.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
export BENCH_AB="X=1;PCOPS_FPS_MW=0;X=1;PCOPS_FPS_MW=0"
bash tools/gpu_run.sh $O bench_ab || exit 1
grep -E '^==|ms_per_step' $O/bench_ab.txt | sed 's/.*"ms_per_step": \([0-9.]*\).*/\1/' | paste - -
for v in X=1 PCOPS_FPS_MW=0 X=1 PCOPS_FPS_MW=0; do
  echo "== $v" >> $O/ps.txt
  env $v timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline --no-fp32-leg --no-extra-legs --no-kernel-timing --steps 20 --warmup 3 >> $O/ps.txt 2>> $O/ps.err || exit 1
done
grep -E '^==|ms_per_step' $O/ps.txt | sed 's/.*"ms_per_step": \([0-9.]*\).*/\1/' | paste - -
