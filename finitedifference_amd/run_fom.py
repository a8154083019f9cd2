"""Run the full-order model and save the HDM snapshots (drop-in for
C/run_fom.py:9-52 of the reference; F/run_fom.py and T/run_fom.py differ
only in the grid size and return value, exposed here as keywords)."""
import time

import numpy as np

from .dist import job
from .hypernet2D import load_or_compute_snaps, make_2D_grid


def main(mu1=5.19, mu2=0.026, save_snaps=True, *, num_cells=250, num_steps=500, dt=0.05,
         snap_folder="param_snaps", return_snaps=True, **solver_kw):
    """Same flow as the reference: 250^2 grid on [0,100]^2, dt=0.05, 500
    steps, w0 = 1, cached through load_or_compute_snaps; timed region as
    C/run_fom.py:41-43.  Returns (elapsed, snaps) like the Coarse driver
    (return_snaps=False gives the Fine/TestAE drivers' (elapsed, 0)).
    Under torchrun (one process per GPU) every rank runs its row slab and
    gets the whole matrix (load_or_compute_snaps); rank 0 prints and saves."""
    num_cells_x, num_cells_y = num_cells, num_cells
    xl, xu, yl, yu = 0, 100, 0, 100
    grid_x, grid_y = make_2D_grid(xl, xu, yl, yu, num_cells_x, num_cells_y)
    u0 = np.ones((num_cells_y, num_cells_x))
    v0 = np.ones((num_cells_y, num_cells_x))
    w0 = np.concatenate((u0.flatten(), v0.flatten()))
    mu_rom = [mu1, mu2]
    t0 = time.time()
    hdm_snaps = load_or_compute_snaps(mu_rom, grid_x, grid_y, w0, dt, num_steps,
                                      snap_folder=snap_folder, **solver_kw)
    elapsed_time = time.time() - t0
    # multi-GPU job (torchrun): every rank ran its slab; one of them reports
    # and saves (the reference is one process)
    _, rank, _ = job()
    if rank == 0:
        print(f"Elapsed FOM time: {elapsed_time:.3e} seconds")
    if save_snaps and rank == 0:
        np.save(f"hdm_snaps_mu1_{mu_rom[0]:.2f}_mu2_{mu_rom[1]:.3f}.npy", hdm_snaps)
        print(f"HDM snapshots saved as hdm_snaps_mu1_{mu_rom[0]:.2f}_mu2_{mu_rom[1]:.3f}.npy")
    return elapsed_time, (hdm_snaps if return_snaps else 0)


if __name__ == "__main__":
    main()
