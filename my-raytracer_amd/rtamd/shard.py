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

    def __init__(self, height, width, stripe_h, n, rank, device, dtype=torch.float32, channels=3, frames=0,
                 host_staged=False):
        """host_staged: device buffers go through host memory (gloo rehearsal of the RCCL path)."""
        self.n, self.rank = n, rank
        self.host_staged = host_staged
        self.rows = max_rows(height, stripe_h, n)
        self.ids = [torch.as_tensor(shard_rows(height, stripe_h, n, r), device=device) for r in range(n)]
        lead = (frames,) if frames else ()
        self.row_dim = 1 if frames else 0
        shape = lead + (self.rows, width, channels)
        gdev = "cpu" if host_staged else device
        self.gather_list = [torch.empty(shape, dtype=dtype, device=gdev) for _ in range(n)] if rank == 0 else None
        self.image = torch.empty(lead + (height, width, channels), dtype=dtype, device=device) if rank == 0 else None

    def __call__(self, buf):
        """buf: this rank's packed stripes; with frames == F it may hold the first nf <= F
        frames only ([nf, max_rows, W, C]): just those are sent, and the first nf frames of
        the returned image are valid."""
        d = self.row_dim
        if self.n == 1:
            return buf.narrow(d, 0, self.ids[0].numel())
        glist, image = self.gather_list, self.image
        if self.rank == 0:
            if d == 1 and buf.shape[0] < glist[0].shape[0]:
                nf = buf.shape[0]
                glist = [g[:nf] for g in glist]
                image = image[:nf]
            if buf.shape != glist[0].shape:
                raise ValueError("buffer shape does not match the gather")
        dist.gather(buf.cpu() if self.host_staged else buf, glist, dst=0)
        if self.rank == 0:
            for r in range(self.n):
                part = glist[r].narrow(d, 0, self.ids[r].numel()).to(image.device)
                image.index_copy_(d, self.ids[r], part)
        return image


class PeerFrames:
    """Frame assembly without a gather (RT_FLAG_GLOBAL_ROWS): rank 0 owns `slots` sets of whole
    frames [frames, H, W, C]; every other rank maps them into its address space (rt_ipc_open: IPC
    handles sent once with broadcast_object_list; peer access over xGMI) and its render launches
    write their stripes straight to their global rows there, as pixels finish -- the transfer
    overlaps the render, and there is neither a copy nor a re-interleave.  A launch's frames are
    complete on rank 0 after fence(): a one-element all_reduce on the launch stream of every rank
    (RCCL with "nccl"), which starts after that rank's render in stream order, so rank 0's stream
    passes it only when every rank's render has ended (its waves release their image stores at
    system scope before they exit).  With frames == 0 the buffers are single images [H, W, C].
    Reuse: a rank's next launch into a slot waits only for that slot's previous fence, not for
    what rank 0 does with the frames after it -- a consumer on rank 0 (a copy, an encoder) must be
    done with slot s before any rank launches into s again: give every rank a second fence() after
    the consumer, or enough slots that the consumer ends first (bench.py consumes nothing)."""

    def __init__(self, height, width, n, rank, device, frames=0, slots=1, dtype=torch.float32, channels=3):
        from . import ipc_handle, ipc_open   # librt_hip (lazy: importing this module needs no GPU)
        self.n, self.rank, self.slots = n, rank, slots
        lead = (frames,) if frames else ()
        self.frame_elems = height * width * channels
        self.elem = torch.empty((), dtype=dtype).element_size()
        self.images = [torch.zeros(lead + (height, width, channels), dtype=dtype, device=device)
                       for _ in range(slots)] if rank == 0 else None
        dev = torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()
        handles = [None]
        if rank == 0:
            try:   # the handles, and rank 0's device (every rank sees the node's GPUs with the same ids)
                handles = [([ipc_handle(im.data_ptr()) for im in self.images], dev)]
            except Exception as e:   # every rank learns of it (no rank left waiting in the broadcast)
                handles = [f"rank 0: {e!r}"]
        if n > 1:
            dist.broadcast_object_list(handles, src=0)
        if isinstance(handles[0], str):
            raise RuntimeError(f"PeerFrames: exporting the frame buffers failed ({handles[0]})")
        self._opened = []
        if rank == 0:
            self.base = [im.data_ptr() for im in self.images]
        else:
            self.base = []
            exported, owner = handles[0]
            for h, off in exported:
                ptr = ipc_open(h, off, dev, owner)
                self._opened.append((ptr, off))
                self.base.append(ptr)
        self.flag = torch.zeros(1, dtype=torch.float32, device=device)

    def outs(self, slot, nf):
        """Device pointers (valid in this process) of frames 0..nf of buffer set `slot`."""
        step = self.frame_elems * self.elem
        return [self.base[slot] + f * step for f in range(nf)]

    def fence(self):
        """On the current stream: every rank's work enqueued so far on its launch stream has ended."""
        if self.n > 1:
            dist.all_reduce(self.flag)

    def image(self, slot):
        return self.images[slot] if self.rank == 0 else None

    def close(self):
        from . import ipc_close
        for ptr, off in self._opened:
            ipc_close(ptr, off)
        self._opened = []


def segments(rows):
    """Runs of consecutive global rows in a shard's packed row list: [(first, last) local index]."""
    rows = np.asarray(rows)
    if rows.size == 0:
        return []
    cut = np.flatnonzero(np.diff(rows) != 1) + 1
    starts = np.concatenate([[0], cut])
    ends = np.concatenate([cut, [rows.size]]) - 1
    return list(zip(starts.tolist(), ends.tolist()))


class HaloExchange:
    """Halo rows for the sharded adaptive pass (rt_launch_adaptive_shard).

    The neighbour test of a stripe's first / last row needs the primary colour of the row
    just below / above it, which another rank rendered.  Every such row is the first or
    last row of that rank's stripe, so each rank contributes its stripes' edge rows
    ([2 * segments, W, 3] fp64, padded to the largest rank) to ONE all_gather (RCCL over
    xGMI with "nccl"; at 1080p / 16-row stripes 136 rows = 6.3 MB in all), then picks its
    halo [2 * segments, W, 3] out of the gathered edges in the order
    rt_adaptive_halo_rows lists (halo_rows, from the library).  The only data-path
    exchange besides the final frame gather."""

    def __init__(self, height, width, stripe_h, n, rank, halo_rows, device, dtype=torch.float64, host_staged=False):
        self.n, self.rank = n, rank
        self.host_staged = host_staged
        self.segs = [segments(shard_rows(height, stripe_h, n, r)) for r in range(n)]
        self.max_edges = 2 * max(len(s) for s in self.segs)
        own = self.segs[rank]
        self.edge_index = torch.tensor([i for a, b in own for i in (a, b)], dtype=torch.long, device=device)
        where = {}   # global row -> flat index into the gathered edges
        for r in range(n):
            rows = shard_rows(height, stripe_h, n, r)
            for k, (a, b) in enumerate(self.segs[r]):
                where[int(rows[a])] = r * self.max_edges + 2 * k
                where[int(rows[b])] = r * self.max_edges + 2 * k + 1
        missing = [int(y) for y in halo_rows if y >= 0 and int(y) not in where]
        if missing:
            raise ValueError(f"halo rows {missing[:4]} are not edge rows of any shard")
        self.pick = torch.tensor([where.get(int(y), 0) for y in halo_rows], dtype=torch.long, device=device)
        self.send = torch.zeros((self.max_edges, width, 3), dtype=dtype, device=device)
        self.recv = [torch.empty_like(self.send) for _ in range(n)]

    def __call__(self, prim):
        """prim: this rank's packed primary rows [rows, W, 3] (fp64) -> halo [2 * segments, W, 3]."""
        k = self.edge_index.numel()
        self.send[:k].copy_(prim.index_select(0, self.edge_index))
        if self.n == 1:
            return self.send.index_select(0, self.pick)
        if self.host_staged:   # gloo rehearsal: host copies
            recv = [t.cpu() for t in self.recv]
            dist.all_gather(recv, self.send.cpu())
            return torch.cat(recv, 0).to(self.send.device).index_select(0, self.pick)
        dist.all_gather(self.recv, self.send)
        return torch.cat(self.recv, 0).index_select(0, self.pick)
