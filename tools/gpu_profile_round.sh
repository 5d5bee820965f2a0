#!/bin/bash
# One GPU session: full bench line, rocprofv3 kernel-trace summary of the same
# command, and two PMC passes (FETCH_SIZE / WRITE_SIZE) for HBM traffic.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
OUT=${1:-gpurun_out/round}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && echo bench ok &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_traced.json 2> $OUT/trace.err && echo trace ok &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'attn_|ln_|fps_|chamfer_|knn|colsum|pcsa' --output-format csv \
  -d $OUT/pmc_fetch -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing \
  > /dev/null 2> $OUT/pmc_fetch.err && echo fetch ok &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'attn_|ln_|fps_|chamfer_|knn|colsum|pcsa' --output-format csv \
  -d $OUT/pmc_write -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing \
  > /dev/null 2> $OUT/pmc_write.err && echo write ok &&
timeout -k 10 400 python bench.py --model pointsea > $OUT/bench_pointsea.json 2> $OUT/bench_pointsea.err && echo pointsea ok
