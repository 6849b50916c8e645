#!/usr/bin/env bash
# Round 6: fewer, larger launches for the headline (explicit batch 1364 / 2047 spp against the
# budget's 682): whole job and cold end to end (the first frame allocates the larger slabs).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06r
for spec in "b0|0" "b1364|1364" "b2047|2047" "b0x|0" "b1364x|1364" "b2047x|2047"; do
  IFS='|' read -r name b <<< "$spec"
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --batch $b > gpurun_out/r06r/$name.json 2> gpurun_out/r06r/$name.log || { tail -5 gpurun_out/r06r/$name.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['end_to_end']; print('%-7s whole %.0f kernel %.0f launch %.2f ms  cold %.0f (%.3f s, frame %.3f s)' % (sys.argv[2], d['value'], d['kernel_mrays'], d['roofline']['avg_launch_ms'], e['value'], e['seconds'], e['frame_with_d2h_s']))" gpurun_out/r06r/$name.json $name
done
