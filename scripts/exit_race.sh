#!/usr/bin/env bash
# A one-shot small render that exits while the scene kernel's hipRTC compile may still be
# running (fresh code-object cache each run): the exit code of each of N runs (0 expected).
# usage: bash scripts/exit_race.sh N [env...]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
N=$1; shift
code="import sys, json; sys.path.insert(0, '$R/pathtracer-cpp_amd'); import ptamd; from ptamd import scenes; \
sc = scenes.cornell((16, 16)); img, st = ptamd.render(ptamd.Camera.from_spec(sc.camera), ptamd.BVH.from_scene(sc), 2, 5); \
print(st['kernel_path'])"
bad=0
for i in $(seq 1 "$N"); do
  d=$(mktemp -d)
  timeout -k 5 60 env PT_RTC_CACHE_DIR="$d" "$@" python3 ${PY_FLAGS:--X faulthandler} -c "$code" > /tmp/er_out.txt 2> /tmp/er_err.txt
  rc=$?
  echo "run $i rc=$rc out=$(tr -d '\n' < /tmp/er_out.txt)"
  if [ $rc -ne 0 ]; then bad=$((bad + 1)); grep -v amdgpu.ids /tmp/er_err.txt | tail -30; fi
  rm -rf "$d"
done
echo "nonzero exits: $bad of $N"
