set -o pipefail
O=gpurun_out/r1s12; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo bench ok &&
timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/bench_ps.json 2> $O/bench_ps.err && echo psbench ok
