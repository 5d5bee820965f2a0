set -o pipefail
O=gpurun_out/r4j; mkdir -p $O
export PYTEST_K="add_posemb or cd_l1_parity"; bash tools/gpu_run.sh $O tests_k || exit 1
cp tuning/tunableop_svdformer_gfx950.csv $O/tunableop_svdformer_gfx950.prev.csv
timeout -k 10 900 python bench.py --tunableop tune --steps 2 --warmup 1 --no-cpu-baseline --no-extra-legs --no-kernel-timing --no-fp32-leg > $O/tune.json 2> $O/tune.err || exit 1
cp tuning/tunableop_svdformer_gfx950.csv $O/tunableop_svdformer_gfx950.csv
timeout -k 10 400 python bench.py --no-cpu-baseline --no-extra-legs --no-fp32-leg > $O/bench_newtune.json 2> $O/bench_newtune.err || exit 1
cp $O/tunableop_svdformer_gfx950.prev.csv tuning/tunableop_svdformer_gfx950.csv
timeout -k 10 400 python bench.py --no-cpu-baseline --no-extra-legs --no-fp32-leg > $O/bench_oldtune.json 2> $O/bench_oldtune.err
timeout -k 10 120 python tools/knn_bench.py > $O/knn_base.txt 2>&1
PCOPS_LIB_PATH=$PWD/tools/ab/libpcops_knnabl.so timeout -k 10 120 python tools/knn_bench.py > $O/knn_ablation.txt 2>&1
