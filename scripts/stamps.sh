#!/usr/bin/env bash
# In-kernel s_memtime section stamps (diagnostic library lib/libpt_hip_stamps.so, built
# here by `make -C pathtracer-cpp_amd stamps`): one short bench run per scene, the
# [stamps] lines of the render go to gpurun_out/stamps/<name>.log.
# usage: bash scripts/stamps.sh "NAME|ENV=VAL ...|bench args" ...
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/stamps
for spec in "$@"; do
  IFS='|' read -r name envs args <<< "$spec"
  timeout -k 10 300 env PT_TEST_HOOKS=1 PT_LIB="$R/pathtracer-cpp_amd/lib/libpt_hip_stamps.so" \
      PT_RTC_DEFINES=PT_STAMPS=1 $envs python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e $args \
      > gpurun_out/stamps/$name.json 2> gpurun_out/stamps/$name.log
  rc=$?
  if [ $rc -ne 0 ]; then echo "stamps $name rc=$rc"; tail -5 gpurun_out/stamps/$name.log; exit $rc; fi
  echo "== $name"; grep "\[stamps\]" gpurun_out/stamps/$name.log | tail -3
done
