set -o pipefail
O=gpurun_out/r1s37; mkdir -p $O
for i in 1 2; do
timeout -k 10 300 env PCOPS_FLATGRAD=preset python bench.py --no-cpu-baseline --no-kernel-timing > $O/pre$i.json 2> $O/pre$i.err && echo pre$i ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing > $O/cat$i.json 2> $O/cat$i.err && echo cat$i ok || exit 1
done
timeout -k 10 400 env MIOPEN_FIND_MODE=1 python bench.py --no-cpu-baseline --no-kernel-timing > $O/find1.json 2> $O/find1.err && echo find1 ok
