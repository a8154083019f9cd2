"""Row-slab decomposition over GPUs (one process per GPU, RCCL over xGMI).

Rank k owns the contiguous global rows [row0_k, row0_k + rows_k) of the
nx x ny grid (rows split as evenly as possible, remainder to the first
ranks, e.g. 750 over 8 = 94,94,94,94,94,94,93,93).  The upwind march couples
a slab only to the row just below it, so the exchange is one-way
(rank k -> k+1) and happens inside libburgers_hip over RCCL.
"""
from .solver import FOMContext


def slab_rows(ny, world, rank):
    base, extra = divmod(ny, world)
    rows = base + (1 if rank < extra else 0)
    row0 = rank * base + min(rank, extra)
    return row0, rows


def make_slab_context(nx, ny, rank=0, world=1, device=0, **opts):
    if world == 1:
        return FOMContext(nx, ny, device, **opts)
    return FOMContext.slab(nx, ny, rank, world, device, **opts)
