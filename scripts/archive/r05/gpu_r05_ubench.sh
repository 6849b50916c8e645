#!/usr/bin/env bash
# Round 5: the VALU issue peak against MI355X_MICROARCH.md's "v_fma_f32 wave64: 2 cyc
# (SIMD-32); one wave alone: 4": tools/valu_ubench at 1, 2, 4 and 8 waves per SIMD for
# v_fma_f32, v_pk_fma_f32, v_add_f32, v_max3_f32 (+ mul, fma+add), then one PMC pass at 8
# waves for the second-port share (SQ_ACTIVE_INST_VALU2). -> gpurun_out/r05_ubench/
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05_ubench"; mkdir -p "$O"
B="$R/pathtracer-cpp_amd/bin/valu_ubench"
OPS="fma pk_fma add max3 mul fma+add"
for w in 1 2 4 8; do
  timeout -k 10 120 "$B" $w $OPS > "$O/ubench_w$w.txt" 2>&1 || { echo "ubench w$w failed"; cat "$O/ubench_w$w.txt"; exit 1; }
  cat "$O/ubench_w$w.txt"
done
cd /tmp && export TMPDIR=/tmp
for w in 1 8; do
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE \
  -d "$O/pmc_w$w" -o pmc --output-format csv -- "$B" $w $OPS > "$O/pmc_w$w.log" 2>&1 || { echo "pmc w$w failed"; tail -5 "$O/pmc_w$w.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$O/kt_w$w" -o kt --output-format csv -- "$B" $w $OPS > "$O/kt_w$w.log" 2>&1 || { echo "kt w$w failed"; exit 1; }
done
echo "ubench done"
