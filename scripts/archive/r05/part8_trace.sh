set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/p8
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/p8/kt" -o kt --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --part 0/8 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > "$GRAFT_REPO_ROOT/gpurun_out/p8/b.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/p8/b.log"
rc=$?; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/p8/b.log"; exit $rc
