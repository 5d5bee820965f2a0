# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5kq; mkdir -p $O
for r in 1 2 3; do
  for kp in 0 16777216 67108864; do
    if [ $kp = 0 ]; then E="X=0"; else E="HSA_KERNARG_POOL_SIZE=$kp"; fi
    echo "== $E" >> $O/ab.txt
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --no-extra-legs --no-kernel-timing --steps 30 --warmup 3 >> $O/ab.txt 2>> $O/ab.err || exit 1
  done
done
python - <<'PY'
import json
for l in open('gpurun_out/r5kq/ab.txt'):
    if l.startswith('=='): print(l.strip(), end=' ')
    elif l.startswith('{'):
        d=json.loads(l); print(round(d['ms_per_step'],2), 'host', round(d.get('host_issue_ms_per_step',0),2))
PY
