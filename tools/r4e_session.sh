# ST tile-pipeline A/B: bitwise equality (attn_variant) and timing (attn_bench) per kernel
set -o pipefail
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 300 python tools/attn_variant.py dump $O/base.pt > $O/variant_base.txt 2>&1 || exit 1
PCOPS_FWD_ST=1 PCOPS_DQ_ST=1 PCOPS_DKV_ST=1 timeout -k 10 300 python tools/attn_variant.py dump $O/st.pt > $O/variant_st.txt 2>&1 || exit 1
python tools/attn_variant.py cmp $O/base.pt $O/st.pt > $O/variant_cmp.txt 2>&1
rm -f $O/base.pt $O/st.pt
for i in 1 2; do
  timeout -k 10 300 python tools/attn_bench.py 0 1 2 3 > $O/bench_base_$i.txt 2>&1 || exit 1
  PCOPS_FWD_ST=1 PCOPS_DQ_ST=1 PCOPS_DKV_ST=1 timeout -k 10 300 python tools/attn_bench.py 0 1 2 3 > $O/bench_st_$i.txt 2>&1 || exit 1
done
