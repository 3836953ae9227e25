"""Row-stripe sharding of one frame over the GPUs of a node (one process per GPU).

Rank r renders the rows y with (y // stripe_h) % n == r (interleaved stripes
balance the per-row cost), packed in increasing y (rt_render_params rules).
The frame is assembled on rank 0 by ONE collective: torch.distributed.gather
of equal-sized (padded) stripe buffers -- RCCL over xGMI with the "nccl"
backend, where every non-root rank sends its buffer on its own link to the
root -- followed by an index_copy that re-interleaves the rows.  There is no
other data-path communication: pixels are independent (mytracer_gpu.cu:132-159).
"""
import numpy as np
import torch
import torch.distributed as dist


def shard_rows(height, stripe_h, n, r):
    y = np.arange(height)
    return y[(y // stripe_h) % n == r]


def max_rows(height, stripe_h, n):
    return max(len(shard_rows(height, stripe_h, n, r)) for r in range(n))


class StripeGather:
    """Pre-allocated gather of per-rank stripe buffers into whole frames on rank 0.

    frames == 0: buffers are [max_rows, W, C] -> one image [H, W, C].
    frames == F: buffers are [F, max_rows, W, C] (the F frames of one rt_launch_frames launch)
    -> [F, H, W, C] with ONE collective per launch instead of F."""

    def __init__(self, height, width, stripe_h, n, rank, device, dtype=torch.float32, channels=3, frames=0):
        self.n, self.rank = n, rank
        self.rows = max_rows(height, stripe_h, n)
        self.ids = [torch.as_tensor(shard_rows(height, stripe_h, n, r), device=device) for r in range(n)]
        lead = (frames,) if frames else ()
        self.row_dim = 1 if frames else 0
        shape = lead + (self.rows, width, channels)
        self.gather_list = [torch.empty(shape, dtype=dtype, device=device) for _ in range(n)] if rank == 0 else None
        self.image = torch.empty(lead + (height, width, channels), dtype=dtype, device=device) if rank == 0 else None

    def __call__(self, buf):
        d = self.row_dim
        if self.n == 1:
            return buf.narrow(d, 0, self.ids[0].numel())
        if self.rank == 0 and buf.shape != self.gather_list[0].shape:
            raise ValueError("buffer shape does not match the gather")
        dist.gather(buf, self.gather_list, dst=0)
        if self.rank == 0:
            for r in range(self.n):
                self.image.index_copy_(d, self.ids[r], self.gather_list[r].narrow(d, 0, self.ids[r].numel()))
        return self.image
