# A/B of the backward-pass occupancy builds + SQ counters of the default build.
set -o pipefail
O=gpurun_out/attn_occ; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python tools/attn_bench.py > $O/default.txt 2>&1 && echo d ok &&
PCOPS_LIB_PATH=tools/exp/occ_dq/libpcops.so timeout -k 10 120 python tools/attn_bench.py > $O/occ_dq.txt 2>&1 && echo q ok &&
PCOPS_LIB_PATH=tools/exp/occ_all/libpcops.so timeout -k 10 120 python tools/attn_bench.py > $O/occ_all.txt 2>&1 && echo a ok &&
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1; echo listed &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VALU --kernel-include-regex 'attn_' --output-format csv -d $O/pmc1 -o run -- python tools/attn_bench.py 1 > $O/pmc1.log 2>&1 && echo pmc1 ok
