"""Multi-process frame assembly (ptamd.dist) with torch.distributed/gloo on the CPU,
world_size 2 and 3. Each rank renders its row bands with the CPU oracle (the
checker standing in for the GPU kernel, which the -m gpu tests cover) and the
gathered frame must equal the single-process frame bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, band, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    _render_and_gather(rank, world, band, out_path, dict(rank=rank, world_size=world))


def _spawned(rank, world, band, out_path):
    # started by ptamd.dist.spawn_ranks (bench.py --gpus N without a launcher): the
    # rendezvous comes from the torchrun-style environment it sets
    assert os.environ["RANK"] == str(rank) and os.environ["WORLD_SIZE"] == str(world)
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and os.environ["PT_LAUNCHER"] == "spawn"
    _render_and_gather(rank, world, band, out_path, {})


def _render_and_gather(rank, world, band, out_path, init_kw):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "pathtracer-cpp_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    import _oracle as O
    from ptamd import dist as pdist, scenes
    dist.init_process_group("gloo", **init_kw)
    assert dist.get_world_size() == world and dist.get_rank() == rank
    sc = scenes.cornell((24, 37))
    W, H = sc.camera.res

    def render_part(part, parts, b):
        rows = pdist.part_rows(H, part, parts, b)
        out = np.zeros((len(rows), W, 3), np.float32)
        for i, h in enumerate(rows):
            out[i] = O.render(sc, 3, 5, rows=(h, h + 1))[0][0]
        return out

    frame = pdist.gather_with(render_part, H, W, rank, world, band)
    if rank == 0:
        np.save(out_path, frame.numpy())
    else:
        assert frame is None  # gather to rank 0 only
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,band", [(2, 8), (2, 1), (3, 4)])
def test_gather_frame_matches_single_process(tmp_path, world, band):
    import _oracle as O
    from ptamd import scenes
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(world, _free_port(), band, out), nprocs=world, start_method="spawn")
    frame = np.load(out)
    ref, _ = O.render(scenes.cornell((24, 37)), 3, 5)
    assert np.array_equal(frame.view(np.uint32), ref.view(np.uint32))


def test_spawn_ranks_entry_gathers_bit_identical_frame(tmp_path):
    """The entry bench.py uses for --gpus N without a launcher, driven at world 2 on gloo."""
    import _oracle as O
    from ptamd import dist as pdist, scenes
    out = str(tmp_path / "frame.npy")
    pdist.spawn_ranks(_spawned, 2, (8, out))
    frame = np.load(out)
    ref, _ = O.render(scenes.cornell((24, 37)), 3, 5)
    assert np.array_equal(frame.view(np.uint32), ref.view(np.uint32))


def _bench(args, env_extra):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=300)


def test_bench_refuses_launcher_world_mismatch():
    r = _bench(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and r.stdout == ""
    assert "WORLD_SIZE=2" in r.stderr and "--gpus is 1" in r.stderr


def test_bench_refuses_more_gpus_than_visible():
    import torch
    n = torch.cuda.device_count()
    r = _bench(["--gpus", str(n + 1)], {})
    assert r.returncode == 2 and r.stdout == ""
    assert f"--gpus {n + 1} but {n} GPU(s) visible" in r.stderr


def test_row_owner_index_is_a_permutation():
    from ptamd import dist as pdist
    for H, parts, band in [(37, 2, 8), (1024, 8, 8), (5, 8, 1), (4096, 8, 8)]:
        idx, max_rows = pdist.row_owner_index(H, parts, band)
        assert len(set(idx.tolist())) == H
        assert idx.max() < parts * max_rows
