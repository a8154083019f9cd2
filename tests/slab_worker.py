"""One rank of tests/test_gpu_parity.py::test_slab_halo_two_processes_one_gpu
(not a test module): its slab of an N x N grid, T steps from w0 = 1, on
device 0, rendezvous over gloo; writes its slab snapshot matrix."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


SWEEP_MUS = [(4.25, 0.015), (5.19, 0.026), (5.5, 0.03)]


def main():
    N, T, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    sweep = len(sys.argv) > 4 and sys.argv[4] == "sweep"  # mu sweep (burg_sweep) instead
    import torch.distributed as dist
    from finitedifference_amd.dist import make_slab_context, slab_state
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ctx = make_slab_context(N, N, rank, world, device=0, dist=dist)
    g = np.linspace(0, 100, N + 1)
    ctx.set_problem(g, g, 0.05, (5.19, 0.026))
    w0 = slab_state(np.ones(2 * N * N), N, N, rank, world)
    dist.barrier()
    if sweep:
        snaps, st = ctx.sweep(SWEEP_MUS, T, w0=w0)
        assert st["engine"] == 2
        for j, sn in enumerate(snaps):
            np.save(os.path.join(out, f"slab{rank}_mu{j}.npy"), sn)
    else:
        snaps, st, _, _ = ctx.run(w0, T)
        assert st["engine"] == 2
        np.save(os.path.join(out, f"slab{rank}.npy"), snaps)
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
