#!/usr/bin/env bash
# The reference's modified_cornell.cc (six scenes, 1024^2, 10k spp, depth 5), compiled
# unchanged against the drop-in headers (oracle/_ref/dropin_modified_cornell), timed end to
# end on one GPU: contexts created per render (PT_DEVICES_CACHE=0, rounds 1-4) against the
# cached per-device contexts (default, round 5); each run with its own empty code-object
# cache. PNG bytes compared between the two runs.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/dropin_timing"; mkdir -p "$O/fresh" "$O/cached"
B="$R/oracle/_ref/dropin_modified_cornell"
run() {  # name, env...
  local n=$1; shift
  cd "$O/$n" || exit 1
  local t0; t0=$(date +%s.%N)
  timeout -k 10 300 env PT_RTC_CACHE_DIR="$O/$n/rtc" "$@" "$B" out_ > log.txt 2> err.txt || { echo "$n failed"; tail -5 err.txt; exit 1; }
  echo "$n $(python3 -c "import sys; print('%.3f s' % (float(sys.argv[2]) - float(sys.argv[1])))" "$t0" "$(date +%s.%N)")" | tee time.txt
}
run fresh PT_TEST_HOOKS=1 PT_DEVICES_CACHE=0 PT_DEVICES=0
run cached PT_DEVICES=0
for f in "$O"/fresh/out_*.png; do cmp "$f" "$O/cached/$(basename "$f")" || { echo "PNG differs: $f"; exit 1; }; done
echo "PNG bytes identical: $(ls "$O"/cached/out_*.png | wc -l) files"
