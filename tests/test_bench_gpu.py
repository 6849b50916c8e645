"""bench.py's one-line JSON contract on the GPU (the driver parses this line): a short Cornell
run (the headline workload's scene, resolution and depth at 40 spp) with its CPU baseline and
end-to-end passes, checked for every field the contract names and for the values' sanity."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_line_contract():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--spp", "40", "--steps", "2", "--warmup", "1",
                        "--cpu-spp", "1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout  # exactly one JSON line on stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "end_to_end"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["unit"] == "Mray/s" and d["dtype"] == "f32" and d["scaling"] in ("weak", "strong")
    assert d["config"]["workload"] == "cornell_1024x1024_spp40_depth5"
    rays = d["rays_per_step"]
    assert d["value"] > 0 and abs(rays / (d["ms_per_step"] * 1e-3) / 1e6 - d["value"]) < 1e-6 * d["value"]
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "avg_launch_ms", "pmc_key"):
        assert k in rf, k
    assert rf["kernel"].startswith("pt_trace_flat_rtc")
    sys.path.insert(0, ROOT)
    import bench
    keyed = json.load(open(os.path.join(ROOT, "profiles", "pmc", "cornell_1024x1024_depth5.json"))).get("key")
    if keyed == bench.kernel_key():  # the committed PMC pass is this build's: the fraction is reported
        assert rf["frac"] is not None and 0.5 < rf["frac"] < 1.1, rf
        assert rf["achieved"] == pytest.approx(rf["frac"] * rf["peak"])
        assert rf["valu_insts_issue_frac_2cyc_model"] is not None
    cb = d["cpu_baseline"]
    assert cb["cores"] == 1 and cb["kind"] in ("reference", "port") and cb["value"] > 0 and cb["bitexact_vs_gpu"]
    e = d["end_to_end"]
    for k in ("value", "seconds", "device_init_s", "value_with_device_init", "bvh_build_s", "set_scene_s",
              "context_create_s", "frame_with_d2h_s", "warm"):
        assert k in e, k
    assert 0 < e["value_with_device_init"] < e["value"]
    assert "error" not in e["warm"] and e["warm"]["value"] > 0
