# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r5gl; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python tools/glue_sites.py --nodes --rows 50 > $O/glue_nodes.txt 2>&1 || { tail -20 $O/glue_nodes.txt; exit 1; }
timeout -k 10 500 python tools/glue_sites.py --nodes --rows 40 --model pointsea > $O/glue_nodes_ps.txt 2>&1 || exit 1
head -45 $O/glue_nodes.txt
