"""The host half of libpt_hip.so (BVH builder, scene validation and packing incl. the
quantised wide tree, OBJ/MTL parser, PNG writer) and the CPU oracle, built with
AddressSanitizer + UndefinedBehaviorSanitizer (make asan), run through the C-ABI, OBJ
and oracle CPU tests (scripts/sanitize.sh). GPU sanitizers are not available on the
MI355X pool, so this covers host code only."""
import os
import subprocess

import pytest

from conftest import ROOT


def test_host_code_under_asan_ubsan():
    if not os.path.exists(subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True,
                                         text=True).stdout.strip()):
        pytest.skip("gcc's libasan is not installed")
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "sanitize.sh")], capture_output=True, text=True,
                       timeout=1200)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert " passed" in r.stdout and "failed" not in r.stdout
