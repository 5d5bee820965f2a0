set -o pipefail
O=gpurun_out/r4q; mkdir -p $O
export TMPDIR=/tmp
export PYTEST_K="knn"
bash tools/gpu_run.sh $O tests_k || exit 1
for cfg in "1 1" "0 1"; do
  set -- $cfg
  PCOPS_KNN_SEED=$1 PCOPS_KNN_SHARE=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/prof_s$1_h$2 -o run -- python tools/knn_bench.py > $O/knn_s$1_h$2.txt 2>&1 || exit 1
  f=$(find $O/prof_s$1_h$2 -name '*kernel_stats.csv' -print -quit); cp "$f" $O/stats_s$1_h$2.csv
  find $O/prof_s$1_h$2 -name '*kernel_trace.csv' -delete
done
B="--no-cpu-baseline --no-fp32-leg --no-extra-legs"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/pcn_new_$i.json 2> $O/pcn_new_$i.err || exit 1
  PCOPS_LN_G16=0 PCOPS_PS_ROWS=0 timeout -k 10 300 python bench.py $B > $O/pcn_old_$i.json 2> $O/pcn_old_$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/ps_new_$i.json 2> $O/ps_new_$i.err || exit 1
  PCOPS_LOCAL_FPS_FORK=0 timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/ps_old_$i.json 2> $O/ps_old_$i.err || exit 1
done
