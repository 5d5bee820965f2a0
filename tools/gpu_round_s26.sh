set -o pipefail
O=gpurun_out/r1s26; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo bench ok &&
timeout -k 10 200 python bench.py --model pointsea --no-cpu-baseline > $O/ps1.json 2> $O/ps1.err && echo ps1 ok &&
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > $O/bench2.json 2> $O/bench2.err && echo bench2 ok
