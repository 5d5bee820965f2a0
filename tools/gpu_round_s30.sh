set -o pipefail
O=gpurun_out/r1s30; mkdir -p $O
SHAPES=1 timeout -k 10 400 python tools/step_profile.py --rows 80 > $O/prof.txt 2> $O/prof.err && echo prof ok &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && echo bench ok
