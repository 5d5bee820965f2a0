# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run: the PointSea line and replay trace.
set -o pipefail
O=gpurun_out/r5ps; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_run.sh $O bench_ps trace_ps || exit 1
python -c "import json;d=json.load(open('$O/bench_pointsea.json'));print(d['ms_per_step'],d['value'])"
ls $O
