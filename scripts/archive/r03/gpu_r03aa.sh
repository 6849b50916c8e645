# hipRTC kernel switched in between launches (no wait for the compile): GPU suite + end-to-end A/B
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03aa
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03aa/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03aa/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for spec in "sw|" "wait|PT_RTC_SWITCH=0" "sw2|" "wait2|PT_RTC_SWITCH=0" "mc_sw|" "mc_wait|PT_RTC_SWITCH=0"; do
  IFS='|' read -r name envs <<< "$spec"
  args=""; case $name in mc_*) args="--scene mcornell --rough 0.3";; esac
  timeout -k 10 300 env PT_TEST_HOOKS=1 $envs python bench.py --steps 1 --warmup 0 --no-cpu-baseline $args > gpurun_out/r03aa/$name.json 2> gpurun_out/r03aa/$name.log || { echo "$name failed"; tail -3 gpurun_out/r03aa/$name.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print('%-8s e2e %8.0f Mray/s  %.3f s  frame %.3f s  first kernel %s | steady %.0f' % (sys.argv[2], e['value'], e['seconds'], e['frame_with_d2h_s'], e['first_frame_kernel'], d['value']))" gpurun_out/r03aa/$name.json $name
done
