set -o pipefail
O=gpurun_out/r4t; mkdir -p $O
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag -o run -- \
    python tools/knn_bench.py > $O/knn_$tag.txt 2>&1 || return 1
  f=$(find $O/prof_$tag -name '*kernel_stats.csv' -print -quit); cp "$f" $O/stats_$tag.csv
  find $O/prof_$tag -name '*kernel_trace.csv' -delete
}
run full PCOPS_KNN_SHARE=1 || exit 1
run noshare PCOPS_KNN_SHARE=0 || exit 1
run abl1 PCOPS_LIB_PATH=$PWD/abl/knn1/libpcops.so || exit 1
run abl2 PCOPS_LIB_PATH=$PWD/abl/knn2/libpcops.so || exit 1
