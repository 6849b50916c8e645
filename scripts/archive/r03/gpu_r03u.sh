# work-pool refill size vs the radiance slab's write amplification (Cornell): speed + WRITE_SIZE
set -u
cd $GRAFT_REPO_ROOT
V=pathtracer-cpp_amd/lib/variants
STEPS=3 bash scripts/archive/r03/ab_r03.sh chunk "c1024||" "c512|PT_LIB=$V/libpt_hip_c512.so|" "c256|PT_LIB=$V/libpt_hip_c256.so|" "c1024b||" "c512b|PT_LIB=$V/libpt_hip_c512.so|" "c256b|PT_LIB=$V/libpt_hip_c256.so|" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcw_chunk; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for spec in "c1024|" "c512|PT_LIB=$GRAFT_REPO_ROOT/$V/libpt_hip_c512.so" "c256|PT_LIB=$GRAFT_REPO_ROOT/$V/libpt_hip_c256.so"; do
  IFS='|' read -r name envs <<< "$spec"
  timeout -s KILL 300 env PT_TEST_HOOKS=1 $envs rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $OUT/$name -o w --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/$name.json 2> $OUT/$name.log || { echo "$name pmc failed"; tail -5 $OUT/$name.log; exit 1; }
  python3 - $OUT $name <<'PY'
import csv, glob, sys, collections, json
out, name = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(float)
for f in glob.glob(f"{out}/{name}/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "trace" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
b = json.load(open(f"{out}/{name}.json"))
rays = b["rays_per_step"]
print(name, " ".join(f"{k}={v:.4g}" for k, v in sorted(acc.items())), "write B/ray=%.3f" % (acc["WRITE_SIZE"] * 1024 / rays))
PY
done
