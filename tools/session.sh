# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run: the round-5 closing full pass.
set -o pipefail
O=gpurun_out/r5fin2; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_run.sh $O tests smoke bench trace || exit 1
tail -2 $O/pytest_gpu.log; tail -1 $O/smoke.log
python -c "import json;d=json.load(open('$O/bench.json'));print(d['ms_per_step'],d['value'],d['pointsea_train_step'].get('ms_per_step'))"
head -2 $O/trace_window.txt
timeout -k 10 400 python tools/glue_sites.py --nodes > $O/glue_nodes.txt 2> $O/glue_nodes.err || true
