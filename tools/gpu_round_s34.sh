set -o pipefail
O=gpurun_out/r1s35; mkdir -p $O
timeout -k 10 200 python tools/attn_bench.py > $O/attn.log 2>&1 && echo attn ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo bench ok &&
timeout -k 10 200 python bench.py --model pointsea --no-cpu-baseline > $O/ps1.json 2> $O/ps1.err && echo ps1 ok
