#!/usr/bin/env bash
# Round 6: context stream made on a thread + compile started before the upload — GPU suite, cold
# end to end (config 4 x3 and headline x3, each against PT_CTX_SYNC=1), config 4's 8-GPU share's
# fixed per-launch cost (scripts/part_tail.py).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/r06l
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06l/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06l/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --scene sphere --spp 1000 > gpurun_out/r06l/e2e_c4_$i.json 2> gpurun_out/r06l/e2e_c4_$i.log || exit 1
  PT_TEST_HOOKS=1 PT_CTX_SYNC=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --scene sphere --spp 1000 > gpurun_out/r06l/e2e_c4sync_$i.json 2> gpurun_out/r06l/e2e_c4sync_$i.log || exit 1
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r06l/e2e_$i.json 2> gpurun_out/r06l/e2e_$i.log || exit 1
  PT_TEST_HOOKS=1 PT_CTX_SYNC=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r06l/e2e_sync_$i.json 2> gpurun_out/r06l/e2e_sync_$i.log || exit 1
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06l/e2e*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1]); e = d["end_to_end"]
    print(f, "cold %.0f Mray/s (%.3f s) kernel-only %.0f ratio %.3f build %.3f set_scene %.3f s frame %.3f s" % (e["value"], e["seconds"], d["kernel_mrays"], e["value"] / d["kernel_mrays"], e["bvh_build_s"], e["set_scene_s"], e["frame_with_d2h_s"]))
PY
timeout -k 10 300 python3 scripts/part_tail.py --scene sphere --res 1024 --depth 5 --part 0/8 --spp 250 500 1000 2000 4000 > gpurun_out/r06l/part_tail_c4.json 2> gpurun_out/r06l/part_tail_c4.log || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r06l/part_tail_c4.json')); print('c4 part 0/8: %.4f ms/spp, fixed %.3f ms, fixed / 1000 spp %.4f' % (d['ms_per_spp'], d['fixed_ms'], d['fixed_over_1000spp'])); [print(r['spp'], ['%.3f' % k for k in r['kernel_ms']], r['trace_launches']) for r in d['rows']]"
