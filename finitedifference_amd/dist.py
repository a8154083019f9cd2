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
import tempfile

import numpy as np

from .solver import NPY_EXISTING, NPY_GLOBAL, FOMContext


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


# ---- the reference API on a multi-GPU job ---------------
# inviscid_burgers_implicit2D / load_or_compute_snaps / run_fom.main under
# torchrun: one process per GPU, every rank calls the reference function with
# the reference's arguments (the WHOLE grid and w0); each marches its row slab
# and writes its u rows and its v rows straight into ONE .npy file of the
# whole (2 nx ny, ncols) matrix (burg_run_npy_ex, pwrite at the rows' byte
# offsets), which every rank then maps.

def job():
    """(torch.distributed or None, rank, world) of this process.  Under
    torchrun (WORLD_SIZE > 1 in the environment) the default process group is
    initialised on first use if the caller has not done so -- gloo: the
    library moves no snapshot or halo data through it, only barriers, the
    ring-name and file-name broadcasts and the error agreement.  A single
    process: (None, 0, 1)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return None, 0, 1
    import torch.distributed as dist
    if not dist.is_initialized():
        dist.init_process_group("gloo")
    return dist, dist.get_rank(), dist.get_world_size()


def job_device(device=None):
    """The GPU of this rank: `device` if given, else LOCAL_RANK under a
    multi-process job (one process per GPU), else 0."""
    if device is not None:
        return int(device)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return int(os.environ.get("LOCAL_RANK", "0"))
    return 0


_slab_ctxs = {}


def job_context(nx, ny, device, dist, rank, world, **opts):
    """This rank's cached slab context of an nx x ny grid (make_slab_context:
    every rank must come here together the first time).  A context whose
    launch failed is replaced (its halo rings hold stale colours)."""
    key = (int(device), int(nx), int(ny), int(world), int(rank),
           tuple(sorted((k, v) for k, v in opts.items())))
    ctx = _slab_ctxs.get(key)
    if ctx is None:
        ctx = _slab_ctxs[key] = make_slab_context(nx, ny, rank, world, device=device, dist=dist,
                                                  **opts)
    return ctx


def drop_job_context(ctx):
    for k, v in list(_slab_ctxs.items()):
        if v is ctx:
            del _slab_ctxs[k]
            v.close()


def npy_header(m, ncols):
    """The .npy header burg_run_npy writes (and np.save's format 1.0 layout:
    magic, version, little-endian length, the dict padded with spaces to a
    64-byte boundary, newline) of a C-order float64 (m, ncols) array."""
    d = "{'descr': '<f8', 'fortran_order': False, 'shape': (%d, %d), }" % (m, ncols)
    pad = (64 - (10 + len(d) + 1) % 64) % 64
    d = d + " " * pad + "\n"
    return b"\x93NUMPY\x01\x00" + len(d).to_bytes(2, "little") + d.encode("latin1")


def create_npy(path, m, ncols):
    """A (m, ncols) float64 .npy file of the right size, zero-filled (sparse),
    with burg_run_npy's header: the file every rank of a job writes its rows
    into (burg_run_npy_ex with NPY_EXISTING checks the header and size)."""
    hdr = npy_header(m, ncols)
    with open(path, "wb") as f:
        f.write(hdr)
        f.truncate(len(hdr) + 8 * m * ncols)


def agree(dist, err):
    """Every rank learns whether any rank failed: (first error message or
    None).  Collective."""
    msgs = [None] * dist.get_world_size()
    dist.all_gather_object(msgs, None if err is None else f"{type(err).__name__}: {err}")
    bad = [(r, m) for r, m in enumerate(msgs) if m is not None]
    return None if not bad else "; ".join(f"rank {r}: {m}" for r, m in bad)


def slabs_to_npy(ctx, w0, num_steps, path, snap_every, dist, rank, world):
    """Collective: every rank marches its slab of the trajectory from the
    whole-grid initial state w0 and writes its rows into the .npy file `path`
    of the whole (2 nx ny, num_steps // snap_every + 1) matrix, which rank 0
    creates first.  Raises on every rank if any rank failed (the file is then
    removed).  Returns this rank's stats."""
    nx, ny = ctx.nx, ctx.ny_total
    ncols = int(num_steps) // int(snap_every) + 1
    err = None
    if rank == 0:
        try:
            create_npy(path, 2 * nx * ny, ncols)
        except OSError as e:
            err = e
    bad = agree(dist, err)
    if bad:
        raise RuntimeError(f"snapshot file {path}: {bad}")
    st = None
    try:
        st = ctx.run_to_npy(slab_state(w0, nx, ny, rank, world), num_steps, path,
                            snap_every=snap_every, flags=NPY_GLOBAL | NPY_EXISTING)
    except Exception as e:  # noqa: BLE001  (agreed on below, re-raised on every rank)
        err = e
    bad = agree(dist, err)
    if bad:
        drop_job_context(ctx)
        if rank == 0 and os.path.exists(path):
            os.remove(path)
        dist.barrier()
        raise RuntimeError(f"multi-GPU trajectory failed: {bad}")
    return st


def shared_tmp_path(dist, rank, suffix=".npy"):
    """A fresh path every rank of the job agrees on, in BURG_SNAP_DIR or the
    temporary directory: the ranks must share that directory (one node, as
    the slabs' halo rings require: POSIX shared memory and IPC handles)."""
    box = [None]
    if rank == 0:
        d = os.environ.get("BURG_SNAP_DIR") or tempfile.gettempdir()
        box[0] = os.path.join(d, f"burg_snaps_{os.getpid():x}{secrets.token_hex(6)}{suffix}")
    dist.broadcast_object_list(box, src=0)
    return box[0]
