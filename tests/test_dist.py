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
    import sys
    sys.path.insert(0, os.path.join(ROOT, "pathtracer-cpp_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    import _oracle as O
    from ptamd import dist as pdist, scenes
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
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


def test_row_owner_index_is_a_permutation():
    from ptamd import dist as pdist
    for H, parts, band in [(37, 2, 8), (1024, 8, 8), (5, 8, 1), (4096, 8, 8)]:
        idx, max_rows = pdist.row_owner_index(H, parts, band)
        assert len(set(idx.tolist())) == H
        assert idx.max() < parts * max_rows
