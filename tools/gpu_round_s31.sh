set -o pipefail
O=gpurun_out/r1s32; mkdir -p $O
OPS=aten::copy_,aten::add,aten::add_,aten::sum,aten::cat,aten::mul,aten::max,aten::gelu_backward,aten::gelu timeout -k 10 400 python tools/step_profile.py --rows 60 > $O/ops.txt 2> $O/ops.err && echo ops ok
