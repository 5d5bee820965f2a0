# Scratch GPU session for `gpurun -- bash tools/session.sh` (overwritten for each session; the
# stages are tools/gpu_run.sh's).  This is the last one run.
set -o pipefail
O=gpurun_out/r4fin2; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_run.sh $O tests smoke trace bench bench_ps || exit 1
for d in gauss surface; do
  CH_DATA=$d timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
    SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-include-regex 'chamfer_' --output-format csv \
    -d $O/pmc_ch_$d -o run -- python tools/chamfer_bench.py 5 16384x16384 > $O/pmc_ch_$d.log 2>&1 || exit 1
  python tools/pmc_summary.py "$(find $O/pmc_ch_$d -name '*counter_collection.csv' -print -quit)" > $O/pmc_ch_$d.txt || exit 1
done
