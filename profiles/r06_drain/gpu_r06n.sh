#!/usr/bin/env bash
# Round 6: config 4 launch timeline from the diagnostic stamps library (wave start, first and last
# exhaustion of the work, last wave end; s_memrealtime): one share (part 0/8) at 1000 and 250 spp,
# the whole frame at 1000 spp in one launch.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06n
export PT_TEST_HOOKS=1 PT_LIB="$R/pathtracer-cpp_amd/lib/libpt_hip_stamps.so"
timeout -k 10 300 python3 scripts/part_tail.py --scene sphere --res 1024 --depth 5 --part 0/8 --spp 250 1000 --reps 2 > gpurun_out/r06n/tail_part.json 2> gpurun_out/r06n/tail_part.log || { tail -5 gpurun_out/r06n/tail_part.log; exit 1; }
grep "timeline" gpurun_out/r06n/tail_part.log
timeout -k 10 300 python3 scripts/part_tail.py --scene sphere --res 1024 --depth 5 --part 0/1 --spp 1000 --reps 1 --batch 1000 > gpurun_out/r06n/tail_whole.json 2> gpurun_out/r06n/tail_whole.log || { tail -5 gpurun_out/r06n/tail_whole.log; exit 1; }
grep "timeline" gpurun_out/r06n/tail_whole.log
