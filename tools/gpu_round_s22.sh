set -o pipefail
O=gpurun_out/r1s22; mkdir -p $O
timeout -k 10 240 python bench.py --model pointsea --no-cpu-baseline --no-graph --steps 3 --warmup 2 > $O/ps_eager.json 2> $O/ps_eager.err; echo "eager rc=$?"
