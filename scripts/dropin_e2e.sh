#!/usr/bin/env bash
# The reference's cornell_box.cc (1024^2, 10k spp, depth 5: the headline config), compiled
# unchanged against the drop-in headers (oracle/_ref/dropin_cornell_box), timed as a whole
# process from exec to exit (HIP runtime start, BVH build, scene upload, hipRTC compile, frame,
# PNG write): cold (an empty code-object cache) and warm (the same cache again).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/dropin_e2e"; mkdir -p "$O"
B="$R/oracle/_ref/dropin_cornell_box"
for n in cold warm warm2; do
  t0=$(date +%s.%N)
  timeout -k 10 120 env PT_RTC_CACHE_DIR="$O/rtc" PT_DEVICES=0 "$B" "$O/$n.png" > "$O/$n.log" 2> "$O/$n.err" || { echo "$n failed"; tail -5 "$O/$n.err"; exit 1; }
  python3 -c "import sys; t=float(sys.argv[2])-float(sys.argv[1]); print('%s %.3f s  %.0f Mray/s (3.7073e10 rays)' % (sys.argv[3], t, 3.7072726730e10/t/1e6))" "$t0" "$(date +%s.%N)" "$n" | tee -a "$O/times.txt"
done
cmp "$O/cold.png" "$O/warm.png" && echo "PNG identical"
