set -o pipefail
O=gpurun_out/r4d; mkdir -p $O
export PYTEST_K="cd_l1_parity or forward_matches_reference_gpu"
bash tools/gpu_run.sh $O tests_k || exit 1
timeout -k 10 300 python tools/attn_bench.py 1 3 > $O/attn_fused.txt 2>&1 || exit 1
PCOPS_ATTN_FUSED=0 timeout -k 10 300 python tools/attn_bench.py 1 3 > $O/attn_twopass.txt 2>&1 || exit 1
bash tools/r4e_session.sh || exit 1
bash tools/gpu_run.sh $O bench_ps || exit 1
timeout -k 10 400 python bench.py --model pointsea --no-cpu-baseline --no-input-prefetch > $O/bench_ps_noprefetch.json 2> $O/bench_ps_noprefetch.err
