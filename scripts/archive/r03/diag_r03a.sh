#!/usr/bin/env bash
# Round-3 diagnostics (GPU box): VALU-issue calibration of tools/valu_ubench under
# rocprofv3, and the radiance slab's write traffic on config 4 / Cornell with the
# cache-policy experiment builds (lib/variants: nostore, slabnt, accnt, bothnt).
# usage: bash scripts/archive/r03/diag_r03a.sh   -> gpurun_out/r03a/
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r03a"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1; echo "list rc=$?"
have() { grep -q -w "$1" "$OUT/counters.txt"; }
UB="$R/pathtracer-cpp_amd/bin/valu_ubench"
for w in 7 1; do
  timeout -k 10 60 "$UB" $w > "$OUT/ubench$w.txt" 2>&1; rc=$?; fatal $rc ub$w; cat "$OUT/ubench$w.txt"
  timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d "$OUT/ub${w}_kt" -o kt --output-format csv -- "$UB" $w > "$OUT/ub${w}_kt.log" 2>&1; fatal $? ubkt$w
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
    -d "$OUT/ub${w}_pmc" -o pmc --output-format csv -- "$UB" $w > "$OUT/ub${w}_pmc.log" 2>&1; fatal $? ubpmc$w
done
echo "ubench done"
cd "$R"
bench() {  # name env... -- args
  local name=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  timeout -k 10 200 env PT_TEST_HOOKS=1 "${envs[@]}" python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e "$@" \
    > "$OUT/ab_$name.json" 2> "$OUT/ab_$name.log"; local rc=$?; fatal $rc "ab_$name"
  [ $rc -eq 0 ] && python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-14s %9.0f Mray/s  kernel %9.0f  launch %.2f ms' % (sys.argv[2], d['value'], d['kernel_mrays'], d['roofline']['avg_launch_ms']))" "$OUT/ab_$name.json" $name
}
V="$R/pathtracer-cpp_amd/lib/variants"
S4=(--scene sphere --spp 1000)
bench s4_base X=1 -- "${S4[@]}"
bench s4_nostore PT_LIB=$V/libpt_hip_nostore.so -- "${S4[@]}"
bench s4_slabnt PT_LIB=$V/libpt_hip_slabnt.so -- "${S4[@]}"
bench s4_accnt PT_LIB=$V/libpt_hip_accnt.so -- "${S4[@]}"
bench s4_bothnt PT_LIB=$V/libpt_hip_bothnt.so -- "${S4[@]}"
bench c_base X=1 --
bench c_slabnt PT_RTC_DEFINES=PT_SLAB_NT=1 --
bench c_accnt PT_RTC_DEFINES=PT_ACC_NT=1 --
bench c_bothnt PT_RTC_DEFINES=PT_SLAB_NT=1,PT_ACC_NT=1 --
bench c_nostore PT_RTC_DEFINES=PT_EXP_NO_STORE=1 --
echo "ab done"
cd /tmp
WR=""
for c in TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum; do have $c && WR="$WR $c"; done
TCP=""; have TCP_TCC_WRITE_REQ_sum && TCP="TCP_TCC_WRITE_REQ_sum"
pmc() {  # name "counters" env... -- args
  local name=$1 cs=$2; shift 2; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  timeout -s KILL 120 env PT_TEST_HOOKS=1 "${envs[@]}" rocprofv3 --pmc $cs -d "$OUT/pmc_$name" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-e2e "$@" > "$OUT/pmc_$name.json" 2> "$OUT/pmc_$name.log"
  local rc=$?; fatal $rc "pmc_$name"; echo "pmc $name rc=$rc"
}
for v in base slabnt bothnt; do
  lib=(X=1); [ $v != base ] && lib=(PT_LIB=$V/libpt_hip_$v.so)
  pmc s4_${v}_w "WRITE_SIZE" "${lib[@]}" -- "${S4[@]}"
  pmc s4_${v}_f "FETCH_SIZE" "${lib[@]}" -- "${S4[@]}"
  pmc s4_${v}_h "TCC_HIT_sum TCC_MISS_sum" "${lib[@]}" -- "${S4[@]}"
  [ -n "$WR$TCP" ] && pmc s4_${v}_req "$WR $TCP" "${lib[@]}" -- "${S4[@]}"
done
for v in base bothnt; do
  d=(X=1); [ $v = bothnt ] && d=(PT_RTC_DEFINES=PT_SLAB_NT=1,PT_ACC_NT=1)
  pmc c_${v}_w "WRITE_SIZE" "${d[@]}" --
  pmc c_${v}_f "FETCH_SIZE" "${d[@]}" --
  [ -n "$WR$TCP" ] && pmc c_${v}_req "$WR $TCP" "${d[@]}" --
done
echo "diag done"
