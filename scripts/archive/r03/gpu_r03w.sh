# wide walk: XCD-affine work regions (8 bands of rows, one per XCD) vs one region vs HEAD
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03w
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03w/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03w/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
H=pathtracer-cpp_amd/lib/variants/libpt_hip_head.so
S="--scene sphere --spp 1000"
STEPS=3 bash scripts/archive/r03/ab_r03.sh xcd "s_head|PT_LIB=$H|$S" "s_r8||$S" "s_r1|PT_XCD_REGIONS=1|$S" "s_head2|PT_LIB=$H|$S" "s_r8b||$S" "s_r1b|PT_XCD_REGIONS=1|$S" || exit 1
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_xcd; mkdir -p $OUT
for spec in "r8|" "r1|PT_XCD_REGIONS=1"; do
  IFS='|' read -r name envs <<< "$spec"
  timeout -s KILL 300 env PT_TEST_HOOKS=1 $envs rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/$name -o t --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e $S > $OUT/$name.json 2> $OUT/$name.log || { echo "$name pmc failed"; exit 1; }
  python3 - $OUT $name <<'PY'
import csv, glob, sys, collections
out, name = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(float)
for f in glob.glob(f"{out}/{name}/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "trace" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(name, "L2 hit %.4f" % (acc["TCC_HIT_sum"] / (acc["TCC_HIT_sum"] + acc["TCC_MISS_sum"])), dict(acc))
PY
done
