"""World-size-2 gloo test of the row-stripe sharding + gather (CPU).

Each rank renders its interleaved stripes of the cornell frame with the CPU
oracle (no GPU here), then rtamd.shard.StripeGather -- the exact code bench.py
runs over RCCL -- gathers them on rank 0, which must reproduce the full frame
bit for bit, and the per-rank ray counts must add up to the full frame's.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, stripe_h):
    sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle
    import rtamd
    from rtamd.shard import StripeGather

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hs = rtamd.HostScene.generate("cornell")
    hs.prepare()
    orc = pyoracle.Oracle(hs.raw, hs)
    W, H = 64, 45
    p = hs.render_params(W, H, 1)
    p.stripe_height, p.stripe_count, p.stripe_index = stripe_h, world, rank
    part, cnt = orc.render(p, pyoracle.MODE_REFERENCE, threads=1)
    g = StripeGather(H, W, stripe_h, world, rank, device="cpu", dtype=torch.float64)
    buf = torch.zeros((g.rows, W, 3), dtype=torch.float64)
    buf[: part.shape[0]] = torch.from_numpy(part)
    img = g(buf)
    # batched form (one collective for the F frames of a multi-frame launch): frame f = part * (f + 1)
    F = 3
    gb = StripeGather(H, W, stripe_h, world, rank, device="cpu", dtype=torch.float64, frames=F)
    bb = torch.zeros((F, gb.rows, W, 3), dtype=torch.float64)
    for f in range(F):
        bb[f, : part.shape[0]] = torch.from_numpy(part) * (f + 1)
    imgs = gb(bb)
    if rank == 0:
        for f in range(F):
            assert torch.equal(imgs[f], img * (f + 1))
    rays = torch.tensor([cnt.primary_rays + cnt.shadow_rays + cnt.reflection_rays], dtype=torch.float64)
    dist.all_reduce(rays)
    if rank == 0:
        np.save(out_dir / "gathered.npy", img.numpy())
        np.save(out_dir / "rays.npy", rays.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,stripe_h", [(2, 16), (2, 4), (3, 8)])
def test_gloo_stripe_gather_reproduces_full_frame(tmp_path, world, stripe_h):
    mp.spawn(_worker, args=(world, _free_port(), tmp_path, stripe_h), nprocs=world, join=True)
    sys.path.insert(0, str(ROOT / "my-raytracer_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle
    import rtamd

    hs = rtamd.HostScene.generate("cornell")
    hs.prepare()
    full, cnt = pyoracle.Oracle(hs.raw, hs).render(hs.render_params(64, 45, 1))
    assert np.array_equal(np.load(tmp_path / "gathered.npy"), full)
    assert np.load(tmp_path / "rays.npy")[0] == cnt.primary_rays + cnt.shadow_rays + cnt.reflection_rays
