"""Host-side logic mirrored from the reference (CPU only)."""
import os

import numpy as np
import pytest

from finitedifference_amd import grid, hypernet2D as hn
from finitedifference_amd.dist import slab_rows


def test_make_2D_grid_matches_reference_formula():
    gx, gy = grid.make_2D_grid(0, 100, 0, 100, 250, 250)
    assert gx.shape == (251,) and gy[0] == 0 and gy[-1] == 100
    assert np.array_equal(gx, np.linspace(0, 100, 251))


def test_coefficients_are_numpy_rounded_and_reject_nonsquare(orc):
    gx, gy = grid.make_2D_grid(0, 100, 0, 100, 64, 64)
    ix, iy, src, lbc = grid.fom_coefficients(gx, gy, 0.05, (5.19, 0.026))
    P = orc.Problem(64)
    assert np.array_equal(ix, P.inv_dx) and np.array_equal(src, P.src)
    assert np.array_equal(lbc, P.lbc)
    gx2, gy2 = grid.make_2D_grid(0, 100, 0, 100, 7, 5)
    with pytest.raises(ValueError):  # the reference fails the same way
        grid.fom_coefficients(gx2, gy2, 0.05, (5.19, 0.026))
    ix, iy, src, lbc = grid.fom_coefficients(gx2, gy2, 0.05, (5.19, 0.026), allow_nonsquare=True)
    assert lbc.shape == (5,) and np.all(lbc == lbc[0])


def test_param_to_snap_fn_and_cache(tmp_path):
    assert hn.param_to_snap_fn([4.25, 0.015]) == "param_snaps/mu1_4.25+mu2_0.015.npy"
    assert hn.param_to_snap_fn([5.19, 0.026], "x", ".npz") == "x/mu1_5.19+mu2_0.026.npz"
    folder = str(tmp_path / "ps")
    os.makedirs(folder)
    a = np.arange(12.0).reshape(3, 4)
    np.save(hn.param_to_snap_fn([1.0, 2.0], folder), a)
    assert hn.param_to_snap_fn([1.0, 2.0], folder) in hn.get_saved_params(folder)
    got = hn.load_or_compute_snaps([1.0, 2.0], None, None, None, 0.05, 2, snap_folder=folder)
    assert np.array_equal(got, a[:, :3])  # cache hit: np.load(fn)[:, :num_steps+1]


def test_compute_error():
    h = np.random.default_rng(0).random((10, 4)) + 1
    r = h * (1 + 1e-3)
    e, m = hn.compute_error(r, h)
    assert e.shape == (4,) and np.allclose(e, 1e-3 / (1 + 1e-3))


def test_get_ops_is_the_reference_operator_set(orc):
    gx, gy = grid.make_2D_grid(0, 100, 0, 100, 9, 9)
    _, _, JDx, JDy, Eye = hn.get_ops(gx, gy)
    rng = np.random.default_rng(1)
    f = rng.random(81)
    inv = 1.0 / np.diff(gx)
    F = f.reshape(9, 9)
    dx = F * inv[None, :] - np.pad(F * inv[None, :], ((0, 0), (1, 0)))[:, :-1]
    assert np.allclose(JDx @ f, dx.ravel())
    dy = F * inv[:, None] - np.pad(F * inv[:, None], ((1, 0), (0, 0)))[:-1, :]
    assert np.allclose(JDy @ f, dy.ravel())


@pytest.mark.parametrize("ny,world", [(750, 8), (1024, 2), (13, 4), (8192, 4)])
def test_slab_rows_partition(ny, world):
    parts = [slab_rows(ny, world, r) for r in range(world)]
    assert parts[0][0] == 0
    for (a0, n0), (a1, n1) in zip(parts, parts[1:]):
        assert a0 + n0 == a1 and abs(n0 - n1) <= 1
    assert parts[-1][0] + parts[-1][1] == ny


def test_cache_memmap_commit_is_np_save_format(tmp_path):
    """The streamed cache (hypernet2D._open_cache / _commit_cache) produces the
    exact bytes np.save writes for the same array (C/hypernet2D.py:3143)."""
    a = np.random.default_rng(3).random((6, 5))
    fn = str(tmp_path / "mu1_1.0+mu2_2.0.npy")
    tmp, mm = hn._open_cache(fn, 6, 5)
    mm[...] = a
    hn._commit_cache(tmp, fn, mm)
    np.save(str(tmp_path / "ref.npy"), a)
    assert open(fn, "rb").read() == open(str(tmp_path / "ref.npy"), "rb").read()
    assert not os.path.exists(tmp)
