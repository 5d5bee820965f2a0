set -o pipefail
O=gpurun_out/r1s24; mkdir -p $O
timeout -k 10 200 python bench.py --model pointsea --no-cpu-baseline > $O/ps_all.json 2> $O/ps_all.err; echo "all rc=$?"
