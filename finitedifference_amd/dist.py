"""Row-slab decomposition over GPUs (one process per GPU).

Rank k owns the contiguous global rows [row0_k, row0_k + rows_k) of the
nx x ny grid (rows split as evenly as possible, remainder to the first
ranks, e.g. 750 over 8 = 94,94,94,94,94,94,93,93; rank 0 is the bottom slab,
y = 0).  The upwind march couples a slab only to the row just below it
(C/hypernet2D.py:2410-2416: backward differences), so the exchange is
one-way, rank k -> k+1: the north outflow of rank k's top row is the south
inflow of rank k+1's bottom row.  Inside libburgers_hip that stream runs
GPU-to-GPU while both time loops are running, through a ring in the
consumer GPU's memory (producer stores over xGMI) or, as the fallback, in
shared pinned host memory; this module only agrees on
the ring's name, orders context creation, connection and the ring self-test
around barriers, and splits / assembles states and snapshot matrices in the
reference layout.
"""
import os
import secrets

import numpy as np

from .solver import FOMContext


def slab_rows(ny, world, rank):
    base, extra = divmod(ny, world)
    rows = base + (1 if rank < extra else 0)
    row0 = rank * base + min(rank, extra)
    return row0, rows


def slab_state(w, nx, ny, rank, world):
    """This rank's part of a global state w = [u.ravel(), v.ravel()] (u
    row-major (ny, nx), C/run_fom.py:33-35): [u rows | v rows] of the slab."""
    w = np.asarray(w, dtype=np.float64).reshape(2, ny, nx)
    row0, rows = slab_rows(ny, world, rank)
    return np.ascontiguousarray(w[:, row0:row0 + rows, :]).ravel()


def assemble_state(parts, nx, ny):
    """Inverse of slab_state over all ranks (parts in rank order)."""
    world = len(parts)
    out = np.empty((2, ny, nx))
    for r, p in enumerate(parts):
        row0, rows = slab_rows(ny, world, r)
        out[:, row0:row0 + rows, :] = np.asarray(p).reshape(2, rows, nx)
    return out.ravel()


def assemble_snaps(parts, nx, ny):
    """Global snapshot matrix (2*nx*ny, ncols), the reference's layout, from
    per-rank slab snapshot matrices (2*nx*rows_k, ncols)."""
    world = len(parts)
    ncols = parts[0].shape[1]
    out = np.empty((2, ny, nx, ncols))
    for r, p in enumerate(parts):
        row0, rows = slab_rows(ny, world, r)
        out[:, row0:row0 + rows] = np.asarray(p).reshape(2, rows, nx, ncols)
    return out.reshape(2 * ny * nx, ncols)


def agree_halo_name(dist=None):
    """A job-unique ring name, made by rank 0 and broadcast (torch.distributed,
    any backend).  Without a process group: a fresh name (single process)."""
    name = f"{os.getpid():x}{secrets.token_hex(6)}"
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        box = [name]
        dist.broadcast_object_list(box, src=0)
        name = box[0]
    return name


def make_slab_context(nx, ny, rank=0, world=1, device=0, dist=None, halo_name=None, **opts):
    """Context for rank `rank`'s slab.  world > 1: every rank must call this
    together (it creates this rank's inbound halo ring, waits on a barrier
    until all rings exist, attaches the outbound one, and after a second
    barrier checks that the neighbour's probe store crossed the link into a
    device ring -- a failed check moves that boundary to the host ring)."""
    if world == 1:
        return FOMContext(nx, ny, device, **opts)
    if dist is None:
        import torch.distributed as dist
    if halo_name is None:
        halo_name = agree_halo_name(dist)
    row0, rows = slab_rows(ny, world, rank)
    ctx = FOMContext.slab(nx, ny, row0, rows, rank, world, halo_name, device, **opts)
    dist.barrier()
    ctx.connect()
    dist.barrier()
    ctx.verify()
    dist.barrier()
    return ctx


def top_row(w, nx, rows):
    """[u row | v row] of a slab state's top row (the next slab's south halo)."""
    w = np.asarray(w, dtype=np.float64).reshape(2, rows, nx)
    return np.ascontiguousarray(w[:, rows - 1, :]).ravel()


def exchange_halo_rows(rows_up, nx, rank, world, dist, device=None):
    """One-way halo exchange of the row-slab decomposition: rank k sends
    `rows_up` (a float64 array, e.g. the top rows of w and wp) to rank k+1
    and receives rank k-1's (None on rank 0).  torch.distributed send/recv
    (RCCL over xGMI with CUDA tensors when `device` is given, gloo on CPU
    tensors otherwise) -- the exchange step of SURVEY.md section 8(e)."""
    import torch
    dev = torch.device("cuda", device) if device is not None else torch.device("cpu")
    rows_up = np.ascontiguousarray(rows_up, dtype=np.float64)
    got = None
    send = None
    if rank + 1 < world:
        send = torch.from_numpy(rows_up).to(dev)
    if rank > 0:
        got = torch.empty(rows_up.size, dtype=torch.float64, device=dev)
    # even ranks send first, odd ranks receive first: no rank waits on a
    # peer that is itself blocked in a send
    if rank % 2 == 0:
        if send is not None:
            dist.send(send, dst=rank + 1)
        if got is not None:
            dist.recv(got, src=rank - 1)
    else:
        if got is not None:
            dist.recv(got, src=rank - 1)
        if send is not None:
            dist.send(send, dst=rank + 1)
    return None if got is None else got.cpu().numpy()


def slab_residual_norms(ctx, w, wp, dist=None, device=None):
    """Global ||R(w; wp)|| of a row-slab decomposition, every rank passing its
    own slab rows of w and wp: the south halo rows come from the rank below
    (exchange_halo_rows), each rank's sum of squares from burg_slab_residual,
    summed over ranks (all_reduce).  Returns (global norm, this slab's norm).
    Each slab's residual entries equal the single-domain residual's
    (C/hypernet2D.py:2512-2570) bit for bit."""
    nx, rows, rank, world = ctx.nx, ctx.ny, ctx.rank, ctx.world
    if world == 1:
        _, ss = ctx.slab_residual(w, wp)
        return float(np.sqrt(ss)), float(np.sqrt(ss))
    up = np.concatenate((top_row(w, nx, rows), top_row(wp, nx, rows)))
    got = exchange_halo_rows(up, nx, rank, world, dist, device)
    if got is None:
        _, ss = ctx.slab_residual(w, wp)
    else:
        _, ss = ctx.slab_residual(w, wp, got[:2 * nx], got[2 * nx:])
    import torch
    dev = torch.device("cuda", device) if device is not None else torch.device("cpu")
    t = torch.tensor([ss], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return float(np.sqrt(t.item())), float(np.sqrt(ss))
