"""Problem constants (C/config.py:8-27 of the reference)."""
import numpy as np

from .grid import make_2D_grid

BATCH_SIZE = 16
TRAIN_FRAC = 0.9
SNAP_FOLDER = "param_snaps"
SEED = 1234557
DT = 0.05
NUM_STEPS = 500
NUM_CELLS = 250
XL, XU = 0, 100
U0 = np.ones((NUM_CELLS, NUM_CELLS))
V0 = U0.copy()
W0 = np.concatenate((U0.ravel(), V0.ravel()))
GRID_X, GRID_Y = make_2D_grid(XL, XU, XL, XU, NUM_CELLS, NUM_CELLS)
MU1_RANGE = 4.25, 5.5
MU2_RANGE = 0.015, 0.03
SAMPLES_PER_MU = 3


def get_snapshot_params():
    """The 9 training parameters (C/train_autoencoder.py:63-72): mu1 outer,
    mu2 inner, linspace over MU1_RANGE x MU2_RANGE with SAMPLES_PER_MU each."""
    mu1 = np.linspace(MU1_RANGE[0], MU1_RANGE[1], SAMPLES_PER_MU)
    mu2 = np.linspace(MU2_RANGE[0], MU2_RANGE[1], SAMPLES_PER_MU)
    return [[a, b] for a in mu1 for b in mu2]
