#!/bin/bash
# One parameterised GPU session (replaces the round-1 one-off gpu_round_s*.sh):
#   bash tools/gpu_run.sh <out-dir> <stage> [<stage> ...]
# Stages (each under its own time limit; the chain stops at the first failure):
#   tests        pytest -m gpu (thread timeouts, names a hung test)
#   tests_k      pytest -m gpu -k "$PYTEST_K"
#   smoke        __graft_entry__.smoke()
#   probe        tools/valu_probe (VALU issue cost per instruction kind)
#   bench        bench.py default line (PCN, N=1)
#   bench_ps     bench.py --model pointsea
#   bench_fp32   bench.py --fp32 --batch 16 (configs[1] numerics)
#   trace        rocprofv3 --kernel-trace --stats of bench.py
#   pmc_traffic  two PMC passes (FETCH_SIZE / WRITE_SIZE) -> tools/pmc_traffic.py
#   pmc_attn     SQ counter pass over the attention kernels (tools/attn_bench.py)
#   dist1        bench.py under torch.distributed.run with ONE rank and an RCCL group
#                (--dist-selftest): the bucketed all-reduce captured in the graph
#   step_profile tools/step_profile.py (torch-profiler op/kernel breakdown of one eager step)
#   attn_ab      tools/attn_bench.py once per env group in $ATTN_AB (A/B of attention variants)
#   avail        rocprofv3 --list-avail
#   knn          tools/knn_bench.py ; chamfer: tools/microbench.py chamfer
set -o pipefail
OUT=${1:?out dir}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
PMC_RE='attn_|ln_|fps_|chamfer_|knn|colsum|pcsa|gather|group|depth|points2|grid2|transpose_add|bn_|conv3x3|sum_rows|wgrad_skinny|max_k|add_kernel|gelu_bwd'
run_stage() {
  case "$1" in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
             > "$OUT/pytest_gpu.log" 2>&1 ;;
    tests_k) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
             -k "${PYTEST_K:?set PYTEST_K}" > "$OUT/pytest_gpu_k.log" 2>&1 ;;
    smoke) timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 ;;
    probe) timeout -k 10 60 ./tools/valu_probe > "$OUT/valu_probe.txt" 2>&1 ;;
    bench) timeout -k 10 600 python bench.py --detail-json "$OUT/bench_detail.json" ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    bench_ps) timeout -k 10 500 python bench.py --model pointsea --detail-json "$OUT/bench_ps_detail.json" > "$OUT/bench_pointsea.json" 2> "$OUT/bench_pointsea.err" ;;
    bench_sa) PCOPS_CONV1X1=sa timeout -k 10 600 python bench.py --no-cpu-baseline --no-fp32-leg > "$OUT/bench_sa.json" \
             2> "$OUT/bench_sa.err" ;;
    bench_ps_sa) PCOPS_CONV1X1=sa timeout -k 10 500 python bench.py --model pointsea --no-cpu-baseline \
             > "$OUT/bench_pointsea_sa.json" 2> "$OUT/bench_pointsea_sa.err" ;;
    bench_fp32) timeout -k 10 500 python bench.py --fp32 --batch 16 --no-cpu-baseline > "$OUT/bench_fp32.json" \
                  2> "$OUT/bench_fp32.err" ;;
    trace) PCOPS_TRACE_MARKS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
             python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-leg --no-extra-legs \
             > "$OUT/bench_traced.json" 2> "$OUT/trace.err"
           rc=$?
           [ $rc -eq 0 ] && python tools/trace_window.py "$(find "$OUT/trace" -name '*kernel_trace.csv' -print -quit)" 10 \
             "$OUT/kernel_stats_replay.csv" > "$OUT/trace_window.txt" 2>&1
           find "$OUT/trace" -name '*kernel_trace.csv' -exec gzip -9 {} +   # keep the merge-back small
           [ $rc -eq 0 ] || tail -30 "$OUT/trace.err"
           return $rc ;;
    trace_fp32|trace_c1|trace_ps)   # replay-only kernel trace of the fp32 train step / the configs[1] leg / PointSea
      case "$1" in
        trace_fp32) mk=1; tw=5; bargs="--fp32 --steps 5 --warmup 2 --no-extra-legs" ;;
        trace_c1) mk=configs1; tw=3; bargs="--steps 6 --warmup 2 --no-extra-legs --no-kernel-timing" ;;
        trace_ps) mk=1; tw=10; bargs="--model pointsea --steps 10 --warmup 3" ;;
      esac
      PCOPS_TRACE_MARKS=$mk timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$1" -o run -- \
        python bench.py $bargs --no-cpu-baseline > "$OUT/$1.json" 2> "$OUT/$1.err"
      rc=$?
      [ $rc -eq 0 ] && python tools/trace_window.py "$(find "$OUT/$1" -name '*kernel_trace.csv' -print -quit)" $tw \
        "$OUT/${1}_kernel_stats_replay.csv" > "$OUT/${1}_window.txt" 2>&1
      find "$OUT/$1" -name '*kernel_trace.csv' -exec gzip -9 {} +
      [ $rc -eq 0 ] || tail -30 "$OUT/$1.err"
      return $rc ;;
    pmc_traffic|pmc_traffic_ps)
      if [ "$1" = pmc_traffic_ps ]; then M="--model pointsea"; X=_ps; else M=""; X=""; fi
      timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$PMC_RE" --output-format csv \
        -d "$OUT/pmc_fetch$X" -o run -- python bench.py $M --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing \
        --no-fp32-leg --no-extra-legs > /dev/null 2> "$OUT/pmc_fetch$X.err" &&
      timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$PMC_RE" --output-format csv \
        -d "$OUT/pmc_write$X" -o run -- python bench.py $M --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing \
        --no-fp32-leg --no-extra-legs > /dev/null 2> "$OUT/pmc_write$X.err" &&
      python tools/pmc_traffic.py "$(find "$OUT/pmc_fetch$X" -name '*counter_collection.csv' -print -quit)" \
        "$(find "$OUT/pmc_write$X" -name '*counter_collection.csv' -print -quit)" "$OUT/pmc_traffic$X.json" &&
      find "$OUT/pmc_fetch$X" "$OUT/pmc_write$X" -name '*.csv' -exec gzip -9 {} + ;;
    pmc_attn)
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA \
        SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
        --kernel-include-regex 'attn_' --output-format csv -d "$OUT/pmc_attn" -o run -- \
        python tools/attn_bench.py 0 1 > "$OUT/pmc_attn.log" 2>&1 &&
      python tools/pmc_attn.py "$(find "$OUT/pmc_attn" -name '*counter_collection.csv' -print -quit)" \
        > "$OUT/pmc_attn_summary.json" ;;
    pmc_valu)   # VALU counters of the north_star point kernels over the bench's own launches
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
        SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE \
        --kernel-include-regex 'fps_|chamfer_|knn' --output-format csv -d "$OUT/pmc_valu" -o run -- \
        python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-fp32-leg --no-extra-legs \
        > /dev/null 2> "$OUT/pmc_valu.err" &&
      python tools/pmc_valu.py "$(find "$OUT/pmc_valu" -name '*counter_collection.csv' -print -quit)" \
        "$OUT/pmc_valu.json" > "$OUT/pmc_valu.txt" &&
      find "$OUT/pmc_valu" -name '*.csv' -exec gzip -9 {} + ;;
    visited)    # visited pairs of the culled Chamfer on the bench's launches (counting build)
      PCOPS_LIB_PATH=svdformer_pointsea_amd/_lib/count/libpcops.so timeout -k 10 400 \
        python tools/chamfer_visited.py "$OUT/chamfer_visited.json" > "$OUT/chamfer_visited.txt" 2>&1 ;;
    emd)        # EMD timing, bid-pair counts (counting build) and a VALU counter pass over the auction
      timeout -k 10 300 python tools/emd_bench.py "$OUT/emd_bench.json" > "$OUT/emd_bench.txt" 2>&1 &&
      PCOPS_LIB_PATH=svdformer_pointsea_amd/_lib/count/libpcops.so timeout -k 10 300 \
        python tools/emd_bench.py --count "$OUT/emd_pairs.json" >> "$OUT/emd_bench.txt" 2>&1 &&
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
        SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE \
        --kernel-include-regex 'emd_' --output-format csv -d "$OUT/pmc_emd" -o run -- \
        python tools/emd_bench.py "$OUT/emd_bench_pmc.json" > /dev/null 2> "$OUT/pmc_emd.err" &&
      python tools/pmc_valu.py "$(find "$OUT/pmc_emd" -name '*counter_collection.csv' -print -quit)" \
        "$OUT/pmc_emd.json" > "$OUT/pmc_emd.txt" &&
      find "$OUT/pmc_emd" -name '*.csv' -exec gzip -9 {} + ;;
    grad_bisect)  # captured-step gradient report per env group in $BISECT ("A=0;B=0"; "X=1" = the default)
      IFS=';' read -ra groups <<< "${BISECT:?set BISECT}"
      for g in "${groups[@]}"; do
        echo "== $g" >> "$OUT/grad_bisect.txt"
        env $g timeout -k 10 240 python tools/capture_grad_report.py ${BISECT_MODEL:-pointsea} fp32 \
          >> "$OUT/grad_bisect.txt" 2>&1 || return 1
      done ;;
    attn_lib_ab)  # attention A/B of two builds of the library: $AB_BASE (a .so) vs the in-tree one,
                  # attn_bench timings interleaved (base, new, base, new) + a bitwise comparison of outputs
      for i in 1 2; do
        for lib in "${AB_BASE:?set AB_BASE}" ${AB_MORE:-} svdformer_pointsea_amd/_lib/libpcops.so; do
          PCOPS_LIB_PATH=$lib timeout -k 10 180 python tools/attn_bench.py ${ATTN_SHAPES:-0 1 2 3} >> "$OUT/attn_lib_ab.txt" 2>&1 || return 1
        done
      done
      PCOPS_LIB_PATH=$AB_BASE timeout -k 10 300 python tools/attn_variant.py dump "$OUT/av_base.pt" > "$OUT/attn_lib_cmp.txt" 2>&1 &&
      timeout -k 10 300 python tools/attn_variant.py dump "$OUT/av_new.pt" >> "$OUT/attn_lib_cmp.txt" 2>&1 &&
      python tools/attn_variant.py cmp "$OUT/av_base.pt" "$OUT/av_new.pt" >> "$OUT/attn_lib_cmp.txt" 2>&1
      rc=$?; rm -f "$OUT"/av_*.pt; return $rc ;;
    dist1) timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
             --master-port 29611 bench.py --dist-selftest --steps 5 --warmup 2 --no-cpu-baseline --no-fp32-leg --no-extra-legs \
             > "$OUT/bench_dist1.json" 2> "$OUT/bench_dist1.err" ;;
    pmc_attn2)
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS \
        SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC \
        --kernel-include-regex 'attn_' --output-format csv -d "$OUT/pmc_attn2" -o run -- \
        python tools/attn_bench.py 0 1 > "$OUT/pmc_attn2.log" 2>&1 &&
      python tools/pmc_summary.py "$(find "$OUT/pmc_attn2" -name '*counter_collection.csv' -print -quit)" \
        > "$OUT/pmc_attn2_summary.txt" ;;
    attn_ab)   # A/B of attention variants selected by env (ATTN_AB="VAR=a VAR=b;VAR=c" groups)
      IFS=';' read -ra groups <<< "${ATTN_AB:-PCOPS_FWD_PIPE=0}"
      for g in "${groups[@]}"; do
        echo "== $g" >> "$OUT/attn_ab.txt"
        env $g timeout -k 10 120 python tools/attn_bench.py ${ATTN_SHAPES:-0 1 2 3} >> "$OUT/attn_ab.txt" 2>&1 || return 1
      done ;;
    step_profile) timeout -k 10 400 python tools/step_profile.py --rows 60 > "$OUT/step_ops.txt" 2>&1 ;;
    gemm_table) GEMM_TABLE=1 timeout -k 10 400 python tools/op_shapes.py x 60 > "$OUT/gemm_table.txt" 2>&1 ;;
    op_shapes) timeout -k 10 400 python tools/op_shapes.py "${OPS_RE:-^aten::(copy_|cat|fill_|_to_copy)$}" 60 \
                 > "$OUT/op_shapes.txt" 2>&1 ;;
    glue) timeout -k 10 400 python tools/glue_ops.py > "$OUT/glue_ops.txt" 2>&1 &&
          timeout -k 10 400 python tools/glue_ops.py --model pointsea > "$OUT/glue_ops_pointsea.txt" 2>&1 ;;
    bench_ab)  # quick same-box A/B of the PCN step: one short bench per env group in $BENCH_AB ("A=1;A=0")
      IFS=';' read -ra groups <<< "${BENCH_AB:?set BENCH_AB}"
      for g in "${groups[@]}"; do
        echo "== $g" >> "$OUT/bench_ab.txt"
        env $g timeout -k 10 400 python bench.py --no-cpu-baseline --no-fp32-leg --no-extra-legs --no-kernel-timing --steps 20 \
          --warmup 3 >> "$OUT/bench_ab.txt" 2>> "$OUT/bench_ab.err" || return 1
      done ;;
    avail) timeout -k 10 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 ;;
    knn) timeout -k 10 120 python tools/knn_bench.py > "$OUT/knn_bench.txt" 2>&1 ;;
    fps_ab)   # FPS times per env group in $FPS_AB ("A=1;A=0"), default block vs one-wave kernel
      IFS=";" read -ra groups <<< "${FPS_AB:-PCOPS_FPS_WAVE=0;PCOPS_FPS_WAVE=32}"
      for g in "${groups[@]}"; do
        echo "== $g" >> "$OUT/fps_bench.txt"
        env $g timeout -k 10 120 python tools/fps_bench.py >> "$OUT/fps_bench.txt" 2>&1 || return 1
      done ;;
    attn_var)  # bitwise / float64 check of an attention variant: default vs each env group in $ATTN_VAR
      timeout -k 10 300 python tools/attn_variant.py dump "$OUT/attn_var_base.pt" > "$OUT/attn_var.txt" 2>&1 || return 1
      IFS=';' read -ra groups <<< "${ATTN_VAR:?set ATTN_VAR}"
      for g in "${groups[@]}"; do
        echo "== $g" >> "$OUT/attn_var.txt"
        env $g timeout -k 10 300 python tools/attn_variant.py dump "$OUT/attn_var_x.pt" >> "$OUT/attn_var.txt" 2>&1 || return 1
        python tools/attn_variant.py cmp "$OUT/attn_var_base.pt" "$OUT/attn_var_x.pt" >> "$OUT/attn_var.txt" 2>&1
      done
      rm -f "$OUT"/attn_var_*.pt ;;
    attn_det) timeout -k 10 300 python tools/attn_determinism.py > "$OUT/attn_det.txt" 2>&1 ;;
    attn_err) timeout -k 10 300 python tools/attn_err.py > "$OUT/attn_err.jsonl" 2>&1 ;;
    chamfer) timeout -k 10 120 python tools/microbench.py > "$OUT/chamfer_bench.txt" 2>&1 ;;
    *) echo "unknown stage $1"; return 2 ;;
  esac
}
trap 'du -sh "$OUT" 2>/dev/null' EXIT
for s in "$@"; do
  echo "[gpu_run $(date +%T)] $s"
  run_stage "$s" || { rc=$?; echo "[gpu_run] stage $s failed rc=$rc"; exit $rc; }
  echo "[gpu_run $(date +%T)] $s ok"
done
