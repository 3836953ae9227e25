"""Sharded adaptive pass, host side (CPU): the halo rows the library asks for
(rt_adaptive_halo_rows) and their exchange between ranks (rtamd.shard.HaloExchange,
the exact code bench.py runs over RCCL) under gloo with world sizes 2 and 3."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import rtamd
from rtamd.shard import HaloExchange, segments

ROOT = Path(__file__).resolve().parents[1]


def params(W, H, stripe_h=1, count=1, index=0, row_begin=0, row_end=0):
    p = rtamd.abi.RenderParams()
    p.camera.width, p.camera.height = W, H
    p.stripe_height, p.stripe_count, p.stripe_index = stripe_h, count, index
    p.row_begin, p.row_end = row_begin, row_end
    return p


def test_halo_rows_full_frame_and_row_range():
    assert rtamd.adaptive_halo_rows(params(8, 10)).tolist() == [-1, -1]
    assert rtamd.adaptive_halo_rows(params(8, 10, row_begin=3, row_end=7)).tolist() == [2, 7]
    assert rtamd.adaptive_halo_rows(params(8, 10, row_begin=0, row_end=4)).tolist() == [-1, 4]


@pytest.mark.parametrize("H,sh,n", [(45, 16, 2), (45, 8, 3), (10, 1, 4), (37, 5, 8)])
def test_halo_rows_stripes(H, sh, n):
    for r in range(n):
        rows = rtamd.shard_rows(H, sh, n, r)
        hr = rtamd.adaptive_halo_rows(params(8, H, sh, n, r)).tolist()
        segs = segments(rows)
        assert len(hr) == 2 * len(segs)
        for k, (a, b) in enumerate(segs):
            assert hr[2 * k] == (rows[a] - 1 if rows[a] > 0 else -1)
            assert hr[2 * k + 1] == (rows[b] + 1 if rows[b] < H - 1 else -1)
            # each halo row belongs to another rank (interleaved stripes)
            for y in hr[2 * k: 2 * k + 2]:
                if y >= 0 and n > 1:
                    assert (y // sh) % n != r


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, H, W, sh):
    sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
    import rtamd as rt
    from rtamd.shard import HaloExchange as HX

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = torch.from_numpy(np.random.default_rng(7).random((H, W, 3)))
    rows = rt.shard_rows(H, sh, world, rank)
    hr = rt.adaptive_halo_rows(params(W, H, sh, world, rank))
    hx = HX(H, W, sh, world, rank, hr, device="cpu")
    halo = hx(full[torch.as_tensor(rows)].contiguous())
    assert halo.shape == (len(hr), W, 3)
    for i, y in enumerate(hr):
        if y >= 0:
            assert torch.equal(halo[i], full[int(y)]), (rank, i, y)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,H,sh", [(2, 45, 16), (3, 45, 8), (2, 12, 1)])
def test_gloo_halo_exchange(world, H, sh):
    mp.spawn(_worker, args=(world, _free_port(), H, 24, sh), nprocs=world, join=True)


def test_single_rank_halo_is_local():
    H, W = 20, 6
    full = torch.arange(H * W * 3, dtype=torch.float64).reshape(H, W, 3)
    hr = rtamd.adaptive_halo_rows(params(W, H))
    halo = HaloExchange(H, W, 1, 1, 0, hr, device="cpu")(full)
    assert halo.shape == (2, W, 3)
