"""Multi-GPU frame rendering: one process per GPU, rows dealt in bands, one gather.

Partition (the reference's tile loop, render.h:128-139, made static): row h of the
image belongs to rank (h // band) % world. Every rank renders its rows with the
trace kernel into a device tensor; the parts are collected on one rank with a single
`gather` (RCCL over xGMI on MI355X — point-to-point sends to the destination — gloo in
the CPU tests) and interleaved back into the frame on that rank's device. With
per-sample seeding each pixel depends only on (pixel, sample, seed), so the frame is
bit-identical for any world size.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Tuple

import numpy as np


def part_rows(H: int, part: int, parts: int, band: int) -> List[int]:
    """Image rows (h = 0 bottom) owned by `part`, in increasing order."""
    return [h for h in range(H) if (h // band) % parts == part]


def row_owner_index(H: int, parts: int, band: int) -> Tuple[np.ndarray, int]:
    """For the gathered buffer [parts][max_rows] -> image row h; returns (index of
    every image row inside the gathered buffer, max_rows)."""
    rows = [part_rows(H, p, parts, band) for p in range(parts)]
    max_rows = max(len(r) for r in rows)
    index = np.empty(H, dtype=np.int64)
    for p, rs in enumerate(rows):
        for i, h in enumerate(rs):
            index[h] = p * max_rows + i
    return index, max_rows


def gather_frame_to(part, H: int, W: int, rank: int, world: int, band: int, dst: int = 0, group=None):
    """Collect every rank's rows (a contiguous float tensor of rows*W*3 values) on rank
    `dst`: returns the full (H, W, 3) frame there (torch tensor on part's device) and
    None on the other ranks. One gather: each rank sends its max_rows*W*3 block once."""
    import torch
    import torch.distributed as dist
    index, max_rows = row_owner_index(H, world, band)
    rows = len(part_rows(H, rank, world, band))
    send = part.reshape(-1)[: rows * W * 3]
    if rows < max_rows:
        send = torch.cat([send, send.new_zeros((max_rows - rows) * W * 3)])
    if dist.get_backend(group) == "gloo" and send.device.type != "cpu":
        send = send.cpu()  # gloo collectives take host tensors (CPU tests, rehearsals)
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    stacked = torch.stack(bufs).to(part.device).reshape(world * max_rows, W, 3)
    return stacked.index_select(0, torch.as_tensor(index, device=part.device))


def render_distributed(renderer, camera, samples: int, depth: int, rank: int, world: int, band: int = 1,
                       seed: int = 1, group=None, device=None):
    """Render this rank's rows on its GPU (`renderer` = ptamd.Renderer) and gather the
    frame to rank 0. Returns ((H, W, 3) torch tensor on `device` on rank 0, None
    elsewhere; this rank's stats)."""
    import torch
    W, H = camera.res
    rows = len(part_rows(H, rank, world, band))
    dev = device if device is not None else torch.device("cuda", renderer.device)
    part = torch.empty(max(rows, 1) * W * 3, dtype=torch.float32, device=dev)
    torch.cuda.synchronize(dev)
    _, st = renderer.render(camera, samples, depth, seed=seed, part_index=rank, part_count=world, band_rows=band,
                            out=part[: rows * W * 3])
    return gather_frame_to(part[: rows * W * 3], H, W, rank, world, band, 0, group), st


def gather_with(render_part: Callable[[int, int, int], "np.ndarray"], H: int, W: int, rank: int, world: int,
                band: int, group=None):
    """Same collective on any device: `render_part(part, parts, band)` returns this
    rank's rows as an array of shape (rows, W, 3). Used by the gloo (CPU) tests."""
    import torch
    part = torch.as_tensor(np.ascontiguousarray(render_part(rank, world, band), dtype=np.float32))
    return gather_frame_to(part, H, W, rank, world, band, 0, group)


def free_port() -> int:
    """A free TCP port on 127.0.0.1 for the rendezvous of spawned ranks."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_entry(rank: int, fn, world: int, port: int, args: tuple) -> None:
    # torchrun's environment contract, set before anything in this process touches a GPU
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), PT_LAUNCHER="spawn")
    fn(rank, world, *args)


def spawn_ranks(fn, world: int, args: tuple = (), port: Optional[int] = None) -> None:
    """Run fn(rank, world, *args) in `world` fresh processes (one per GPU), each with the
    environment torchrun would give it (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR =
    127.0.0.1, MASTER_PORT), and wait for all of them. The caller must not have touched a
    GPU (the children are started from a fresh interpreter, "spawn"). Raises if any rank
    fails. `fn` must be importable by the children (a module-level function)."""
    import torch.multiprocessing as mp
    mp.start_processes(_rank_entry, args=(fn, world, port or free_port(), args), nprocs=world, join=True,
                       start_method="spawn")
