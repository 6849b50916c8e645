#!/usr/bin/env bash
# Round-3: which VALU forms dual-issue on gfx950 (tools/valu_ubench under rocprofv3,
# SQ_ACTIVE_INST_VALU2), and the fused accumulation's cost on the headline.
# usage: bash scripts/archive/r03/diag_r03c.sh -> gpurun_out/r03c/
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r03c"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
UB="$R/pathtracer-cpp_amd/bin/valu_ubench"
timeout -k 10 90 "$UB" 7 > "$OUT/ubench7.txt" 2>&1; fatal $? ub7; cat "$OUT/ubench7.txt"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d "$OUT/ub_kt" -o kt --output-format csv -- "$UB" 7 > "$OUT/ub_kt.log" 2>&1; fatal $? ubkt
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  -d "$OUT/ub_pmc" -o pmc --output-format csv -- "$UB" 7 > "$OUT/ub_pmc.log" 2>&1; fatal $? ubpmc
echo "ubench done"
cd "$R"
bench() {  # name env... -- args
  local name=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  timeout -k 10 200 env PT_TEST_HOOKS=1 "${envs[@]}" python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e "$@" \
    > "$OUT/ab_$name.json" 2> "$OUT/ab_$name.log"; local rc=$?; fatal $rc "ab_$name"
  [ $rc -eq 0 ] && python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-14s %9.0f Mray/s  kernel %9.0f  launch %.2f ms' % (sys.argv[2], d['value'], d['kernel_mrays'], d['roofline']['avg_launch_ms']))" "$OUT/ab_$name.json" $name
}
bench c_base X=1 --
bench c_noacc PT_RTC_DEFINES=PT_EXP_NO_ACC=1 --
bench c_div1 PT_ACC_DIV=1 --
bench c_div4 PT_ACC_DIV=4 --
bench c_accnt PT_RTC_DEFINES=PT_ACC_NT=1 --
bench c_nostore_noacc PT_RTC_DEFINES=PT_EXP_NO_STORE=1,PT_EXP_NO_ACC=1 --
cd /tmp
timeout -s KILL 200 env PT_TEST_HOOKS=1 PT_RTC_DEFINES=PT_ACC_NT=1 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_c_accnt_w" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > "$OUT/pmc_c_accnt_w.json" 2> "$OUT/pmc_c_accnt_w.log"; fatal $? pmcw
echo "diag done"
