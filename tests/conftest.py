import json
import os
import re
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pathtracer-cpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

GOLDEN = os.path.join(ROOT, "tests", "golden")

# The library honours its test hooks (PT_FLAT, PT_WIDE, PT_PAIRS, ...) only with this gate,
# read once per process when it first looks (pt_internal.h: hook_env).
os.environ.setdefault("PT_TEST_HOOKS", "1")
# Scene setup waits for the scene-specialised (hipRTC) flat kernel, so every flat render in
# the tests runs it; test_rtc_background_compile covers the library default (background
# compile, the generic flat kernel for small renders until it is ready).
os.environ.setdefault("PT_RTC_WAIT", "1")
# The scene kernel's on-disk code-object cache: a fresh directory per test session, so runs
# never read entries an earlier session (or another build) left in the user's cache.
if "PT_RTC_CACHE_DIR" not in os.environ:
    import tempfile
    os.environ["PT_RTC_CACHE_DIR"] = tempfile.mkdtemp(prefix="pt_rtc_cache_")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_meta():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def load_golden(name: str) -> np.ndarray:
    return np.load(os.path.join(GOLDEN, name + ".npy"), allow_pickle=False)


def scene_for(name: str, res):
    """Scene objects for the fixture scene names recorded in golden.json."""
    from ptamd import scenes
    if name == "cornell":
        return scenes.cornell(tuple(res))
    if name == "tri3":
        return scenes.tri3(tuple(res))
    if name.startswith("modified_cornell_r"):
        return scenes.modified_cornell(float(name[len("modified_cornell_r"):]), tuple(res))
    m = re.fullmatch(r"sphere(\d+)_in_cornell", name)
    if m:  # config 4's mesh: sphere223_in_cornell = 99,044 triangles
        return scenes.sphere_in_cornell(int(m.group(1)), tuple(res))
    raise KeyError(name)


def scene_hash(sc) -> str:
    import hashlib
    return hashlib.sha256(sc.with_res(1, 1).to_ptscene().encode()).hexdigest()


@pytest.fixture(scope="session")
def gpu_available():
    import ptamd
    return ptamd.lib().pt_device_count() > 0
