set -o pipefail
mkdir -p gpurun_out/r6h
cp tuning/tunableop_svdformer_gfx950.csv gpurun_out/r6h/old_svdformer.csv
cp tuning/tunableop_pointsea_gfx950.csv gpurun_out/r6h/old_pointsea.csv
timeout -k 10 900 python bench.py --tunableop tune --steps 5 --warmup 2 --no-cpu-baseline --no-fp32-leg --no-extra-legs --no-kernel-timing > gpurun_out/r6h/tune_svd.json 2> gpurun_out/r6h/tune_svd.err
rc=$?; cp tuning/tunableop_svdformer_gfx950.csv gpurun_out/r6h/new_svdformer.csv; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --model pointsea --tunableop tune --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > gpurun_out/r6h/tune_ps.json 2> gpurun_out/r6h/tune_ps.err
rc=$?; cp tuning/tunableop_pointsea_gfx950.csv gpurun_out/r6h/new_pointsea.csv; exit $rc
