"""Host-side latent decoders of the ECSW decoder variants (rom_decoders.py)
against the reference's own decode_* / jac_* outputs at a probe point
(tests/golden/ref_ecsw_variants.npz, made by tests/golden/make_golden.py
from C/hypernet2D.py:1279-1808 and C/rbf_utils.py)."""
import os

import numpy as np
import pytest

import ecsw_models as em
from finitedifference_amd import rom_decoders as rd

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def g():
    return np.load(os.path.join(HERE, "golden", "ref_ecsw_variants.npz"))


@pytest.fixture(scope="module")
def models(g):
    P, Q = g["P"], g["Q"]
    return dict(scaler=em.scaler_of(g["qp_raw"]), kdtree=em.kdtree_of(P),
                gp=em.gp_of(P, Q, *g["gp_par"]))


def rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


def test_scaler_rebuild_matches_fixture(g, models):
    assert np.array_equal(models["scaler"].transform(g["qp_raw"]), g["P"])


@pytest.mark.parametrize("kt", em.RBF_KERNELS_NN)
def test_rbf_nearest_neighbors_decoder(g, models, kt):
    eps, k = float(g["meta"][7]), int(g["meta"][8])
    y, B, B2, P, Q = g["y_probe"], g["basis"], g["basis2"], g["P"], g["Q"]
    w = rd.decode_rbf_nearest_neighbors(y, eps, k, models["kdtree"], P, Q, B, B2,
                                        models["scaler"], kt)
    V = rd.jac_rbf_nearest_neighbors(y, models["kdtree"], P, Q, B, B2, eps, k, models["scaler"], kt)
    assert rel(w, g[f"nn_{kt}_dec"]) <= 1e-14
    assert rel(V, g[f"nn_{kt}_jac"]) <= 1e-14


@pytest.mark.parametrize("kt", em.RBF_KERNELS_GLOBAL)
def test_rbf_global_decoder(g, models, kt):
    eps = float(g["meta"][7])
    y, B, B2, P, Q, W = g["y_probe"], g["basis"], g["basis2"], g["P"], g["Q"], g[f"glob_{kt}_W"]
    w = rd.decode_rbf_global(y, W, P, B, B2, eps, models["scaler"], kt)
    V = rd.jac_rbf_global(y, W, P, Q, B, B2, eps, models["scaler"], kt)
    assert rel(w, g[f"glob_{kt}_dec"]) <= 1e-14
    assert rel(V, g[f"glob_{kt}_jac"]) <= 1e-14


def test_gp_decoder(g, models):
    y, B, B2 = g["y_probe"], g["basis"], g["basis2"]
    assert rel(rd.decode_gp(y, models["gp"], B, B2, models["scaler"]), g["gp_dec"]) <= 1e-12
    # sklearn's own predict path (use_custom_predict=False) gives the same map
    assert rel(rd.decode_gp(y, models["gp"], B, B2, models["scaler"], use_custom_predict=False),
               g["gp_dec"]) <= 1e-12
    assert rel(rd.jac_gp(y, models["gp"], B, B2, models["scaler"]), g["gp_jac"]) <= 1e-12


def test_latent_jacobians_against_differences(g, models):
    """dq/dy of the global gaussian and the GP maps equal central differences
    of q (these two are true derivatives; imq / multiquadric nearest-neighbour
    weights follow the reference's formulas instead, see rom_decoders.py)."""
    y = g["y_probe"]
    for qmap in (rd.RBFGlobalMap(g["glob_gaussian_W"], g["P"], float(g["meta"][7]),
                                 models["scaler"], "gaussian"),
                 rd.GPMap(models["gp"], models["scaler"])):
        J = qmap.dq(y)
        h = 1e-6 * np.maximum(1.0, np.abs(y))
        D = np.stack([(qmap.q(y + h[j] * np.eye(y.size)[j]) - qmap.q(y - h[j] * np.eye(y.size)[j]))
                      / (2 * h[j]) for j in range(y.size)], axis=1)
        assert rel(J, D) <= 1e-6


def test_unsupported_kernels_raise(g, models):
    with pytest.raises(ValueError):
        rd.RBFNearestNeighborsMap(models["kdtree"], g["P"], g["Q"], 1.0, 6, models["scaler"],
                                  "matern")
    with pytest.raises(ValueError):
        rd.RBFGlobalMap(g["glob_gaussian_W"], g["P"], 1.0, models["scaler"], "cubic")
