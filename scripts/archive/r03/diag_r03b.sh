#!/usr/bin/env bash
# Round-3 VALU issue-model calibration (GPU box): the extended tools/valu_ubench (VOP1/2/3,
# VOPC and partial-EXEC forms) under rocprofv3, the trace kernels' VALU mix, and the
# radiance-slab budget A/B on the headline.  usage: bash scripts/archive/r03/diag_r03b.sh -> gpurun_out/r03b/
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r03b"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
UB="$R/pathtracer-cpp_amd/bin/valu_ubench"
timeout -k 10 60 "$UB" 7 > "$OUT/ubench7.txt" 2>&1; fatal $? ub7; cat "$OUT/ubench7.txt"
timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d "$OUT/ub_kt" -o kt --output-format csv -- "$UB" 7 > "$OUT/ub_kt.log" 2>&1; fatal $? ubkt
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d "$OUT/ub_pmc" -o pmc --output-format csv -- "$UB" 7 > "$OUT/ub_pmc.log" 2>&1; fatal $? ubpmc
echo "ubench done"
pmc() {  # name "counters" -- bench args
  local name=$1 cs=$2; shift 3
  timeout -s KILL 200 rocprofv3 --pmc $cs -d "$OUT/pmc_$name" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e "$@" > "$OUT/pmc_$name.json" 2> "$OUT/pmc_$name.log"
  local rc=$?; fatal $rc "pmc_$name"; echo "pmc $name rc=$rc"
}
MIX1="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE"
MIX2="SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_INT64"
pmc c_mix1 "$MIX1" --
pmc c_mix2 "$MIX2" --
pmc s4_mix1 "$MIX1" -- --scene sphere --spp 1000
pmc s4_mix2 "$MIX2" -- --scene sphere --spp 1000
cd "$R"
bench() {  # name env... -- args
  local name=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  timeout -k 10 200 env PT_TEST_HOOKS=1 "${envs[@]}" python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e "$@" \
    > "$OUT/ab_$name.json" 2> "$OUT/ab_$name.log"; local rc=$?; fatal $rc "ab_$name"
  [ $rc -eq 0 ] && python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-14s %9.0f Mray/s  kernel %9.0f  launch %.2f ms' % (sys.argv[2], d['value'], d['kernel_mrays'], d['roofline']['avg_launch_ms']))" "$OUT/ab_$name.json" $name
}
bench c_16g X=1 --
bench c_4g PT_BATCH_BYTES=4294967296 --
bench c_2g PT_BATCH_BYTES=2147483648 --
bench c_16g_again X=1 --
echo "diag done"
