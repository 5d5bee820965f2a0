set -o pipefail
O=gpurun_out/r4ps; mkdir -p $O
export TMPDIR=/tmp
export PYTEST_K="pointsea"
bash tools/gpu_run.sh $O tests_k || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/ps_stream_$i.json 2> $O/ps_stream_$i.err || exit 1
  PCOPS_PS_POINT_STREAM=0 timeout -k 10 300 python bench.py --model pointsea --no-cpu-baseline > $O/ps_serial_$i.json 2> $O/ps_serial_$i.err || exit 1
done
