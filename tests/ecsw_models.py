"""Latent models of the ECSW decoder-variant fixtures (tests/golden/
ref_ecsw_variants.npz), rebuilt from the fixture's arrays: the same
construction in tests/golden/make_golden.py (make_ecsw_variants, which feeds
them to the reference) and in the tests (which feed them to the build).

  scaler   sklearn MinMaxScaler fitted on the training primary coordinates
  kdtree   scipy KDTree over the normalised training set
  gp       GaussianProcessRegressor, ConstantKernel * Matern(nu=1.5), fixed
           hyper-parameters (optimizer=None)
  approx   the NN-decoder stand-in of the rnm variant: a float32 torch map
           y -> U_p y + U_s tanh(A y + b), and jacfwdfunc = torch.func.jacfwd
"""
import numpy as np

RBF_KERNELS_NN = ("gaussian", "imq", "linear", "multiquadric")
RBF_KERNELS_GLOBAL = ("gaussian", "imq", "linear", "multiquadric", "matern")


def scaler_of(qp_raw):
    from sklearn.preprocessing import MinMaxScaler
    return MinMaxScaler().fit(qp_raw)


def kdtree_of(P):
    from scipy.spatial import KDTree
    return KDTree(P)


def gp_of(P, Q, cval, length_scale, alpha):
    from sklearn.gaussian_process import GaussianProcessRegressor
    from sklearn.gaussian_process.kernels import ConstantKernel, Matern
    k = ConstantKernel(cval) * Matern(length_scale=length_scale, nu=1.5)
    return GaussianProcessRegressor(kernel=k, optimizer=None, alpha=alpha).fit(P, Q)


def nn_decoder_of(basis, basis2, A, b):
    import torch
    Up = torch.tensor(basis, dtype=torch.float)
    Us = torch.tensor(basis2, dtype=torch.float)
    At = torch.tensor(A, dtype=torch.float)
    bt = torch.tensor(b, dtype=torch.float)

    def approx(y):
        return Up @ y + Us @ torch.tanh(At @ y + bt)

    jac = torch.func.jacfwd(approx)
    return approx, jac
