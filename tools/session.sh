set -o pipefail
O=gpurun_out/r4h; mkdir -p $O
export PYTEST_K="core_bf16 or attention_bwd_colsum or fused_equals or core_backward_fp32"
bash tools/gpu_run.sh $O tests_k || exit 1
for i in 1 2; do
  ATTN_BENCH_SUMS=1 timeout -k 10 300 python tools/attn_bench.py 0 1 3 > $O/sums_new_$i.txt 2>&1 || exit 1
  ATTN_BENCH_SUMS=1 PCOPS_LIB_PATH=$PWD/tools/ab/libpcops_prev.so timeout -k 10 300 python tools/attn_bench.py 0 1 3 > $O/sums_prev_$i.txt 2>&1 || exit 1
done
timeout -k 10 400 python tools/glue_ops.py > $O/glue_ops.txt 2>&1 || exit 1
bash tools/gpu_run.sh $O trace_fp32 trace_c1
