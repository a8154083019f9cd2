"""Grid and problem coefficients, computed exactly as the reference's NumPy code.

Reference (paths relative to /root/reference, C/ = BurgersFD_CleanCoarse/):
  make_2D_grid            C/hypernet2D.py:2425-2431
  make_ddx spacing 1/dx   C/hypernet2D.py:2410-2416 (np.ones(n) / dx)
  source term             C/hypernet2D.py:2550      dt * 0.02 * exp(mu2 * xc)
  inlet BC                C/hypernet2D.py:2552-2554 lbc[:, 0] = 0.5*dt*mu1**2/dx
"""
import numpy as np


def make_2D_grid(x_low, x_up, y_low, y_up, num_cells_x, num_cells_y):
    """Cell-edge coordinates (C/hypernet2D.py:2425-2431)."""
    grid_x = np.linspace(x_low, x_up, num_cells_x + 1)
    grid_y = np.linspace(y_low, y_up, num_cells_y + 1)
    return grid_x, grid_y


def fom_coefficients(grid_x, grid_y, dt, mu, allow_nonsquare=False):
    """Per-column / per-row coefficient vectors consumed by libburgers_hip.

    Returns (inv_dx[nx], inv_dy[ny], src[nx], lbc[ny]) with NumPy's rounding.
    lbc reproduces the reference's row-indexed quirk ``lbc[:, 0] = ... / dx``
    (row r divides by dx[r]), which only type-checks for nx == ny; like the
    reference, a non-square grid raises ValueError unless
    ``allow_nonsquare=True`` (a performance-only extension that uses dx[0]
    for every row, the value the quirk takes on a uniform grid).
    """
    grid_x = np.asarray(grid_x, dtype=np.float64)
    grid_y = np.asarray(grid_y, dtype=np.float64)
    dx = grid_x[1:] - grid_x[:-1]
    dy = grid_y[1:] - grid_y[:-1]
    xc = (grid_x[1:] + grid_x[:-1]) / 2
    nx, ny = dx.size, dy.size
    inv_dx = np.ones(nx) / dx
    inv_dy = np.ones(ny) / dy
    src = dt * 0.02 * np.exp(mu[1] * xc)
    if nx == ny:
        lbc = 0.5 * dt * mu[0] ** 2 / dx
    elif allow_nonsquare:
        lbc = np.full(ny, 0.5 * dt * mu[0] ** 2 / dx[0])
    else:
        raise ValueError(
            f"could not broadcast input array from shape ({nx},) into shape ({ny},): "
            "the reference FOM (C/hypernet2D.py:2553-2554) requires nx == ny; pass "
            "allow_nonsquare=True for the non-square extension")
    return (np.ascontiguousarray(inv_dx), np.ascontiguousarray(inv_dy),
            np.ascontiguousarray(src), np.ascontiguousarray(lbc))
