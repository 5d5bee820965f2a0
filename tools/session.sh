# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run: the late-round-5 full pass.
set -o pipefail
O=gpurun_out/r5fin; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_run.sh $O tests smoke bench trace || exit 1
tail -3 $O/pytest_gpu.log; cat $O/smoke.log | tail -2
python -c "import json;d=json.load(open('$O/bench.json'));print(d['ms_per_step'],d['value'],d['pointsea_train_step'].get('ms_per_step') if isinstance(d.get('pointsea_train_step'),dict) else None)"
cat $O/trace_window.txt | head -3
