set -o pipefail
O=gpurun_out/r1s6; mkdir -p $O
SHAPES=1 timeout -k 10 300 python tools/step_profile.py --model svdformer --rows 60 > $O/step_svd.txt 2>&1 && echo prof ok
