#!/usr/bin/env bash
# Round 6: fewer, larger fused launches for the headline — the slab budget raised (PT_BATCH_BYTES:
# 32 / 48 GiB -> 1365 / 2047 spp per launch, still two alternating slabs) against the default
# 16 GiB (682 spp): whole job and cold end to end (the first frame allocates the slabs), x2.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06s
for spec in "g16|17179869184" "g32|34359738368" "g48|51539607552" "g16b|17179869184" "g32b|34359738368" "g48b|51539607552"; do
  IFS='|' read -r name bytes <<< "$spec"
  PT_TEST_HOOKS=1 PT_BATCH_BYTES=$bytes timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06s/$name.json 2> gpurun_out/r06s/$name.log || { tail -5 gpurun_out/r06s/$name.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['end_to_end']; print('%-5s whole %.0f kernel %.0f launch %.2f ms step %.2f ms  cold %.0f (%.3f s, frame %.3f s)' % (sys.argv[2], d['value'], d['kernel_mrays'], d['roofline']['avg_launch_ms'], d['ms_per_step'], e['value'], e['seconds'], e['frame_with_d2h_s']))" gpurun_out/r06s/$name.json $name
done
