"""CPU proof of the pipe engine's trajectory-ring indexing (VERDICT r04 item
1a): for every (tile width, steps, snap_every, ring cap) that a GPU test or the
bench runs, burg_ring_audit (host-only, no GPU) replays the ring entries that
ring_load_kernel, the compute waves' store walk (RetCursor), the loader wave's
read walk and ring_extract_kernel form, and checks that

* every entry lies inside the tile's ring (Lt entries: the kernels add
  tile * Lt, so in-range entries of in-range tiles stay inside the allocation;
  the wide steady stores' SGPR offset is not range-checked by the hardware);
* the per-block walks give exactly ring_pos's entry for every diagonal;
* every retained state's cells still hold the diagonal that produced them
  when the launch ends (the retained windows are never overwritten);
* no ring entry is overwritten before the loader wave read it back as the
  previous state (W diagonals later).

The reference keeps every state of a trajectory (C/hypernet2D.py:89-90,126);
these are the states burg_trajectory_copy hands back.
"""
import pytest

from finitedifference_amd import _lib

# (W, num_steps, snap_every, ring_cap): the test_gpu_retained / test_gpu_regime /
# test_gpu_sweep_batch / bench shapes
CASES = [
    (16, 13, 5, 0), (8, 20, 9, 0), (16, 13, 3, 0), (64, 12, 2, 0), (128, 13, 4, 0),
    (256, 11, 2, 0), (1024, 7, 3, 0), (256, 9, 3, 0),          # snap_every windows
    (256, 11, 1, 4), (1024, 12, 1, 5),                          # capped plain rings
    (64, 12, 2, 2), (128, 13, 4, 2), (8, 20, 9, 2), (16, 40, 5, 2), (512, 60, 10, 2),
    (32, 30, 3, 0), (32, 30, 3, 2),                             # shortest working rings
    (256, 500, 1, 0),                                           # bench 4096^2 (W = 256)
    (512, 500, 10, 0), (512, 500, 1, 0),                        # N = 8 slab (16384 x 2048)
    (1024, 500, 10, 0), (1024, 120, 1, 0),                      # 8192^2 (W = 1024)
    (16, 500, 1, 0), (8, 500, 1, 0), (16, 500, 10, 0),          # 1024^2 narrow
]


@pytest.mark.parametrize("W,T,k,cap", CASES)
def test_ring_indices_in_range_and_consistent(W, T, k, cap):
    r = _lib.ring_audit(W, T, k, cap)
    assert r["accesses"] > 64 * W
    assert r["out_of_range"] == 0, r
    assert 0 <= r["max_entry"] < r["entries_per_tile"], r
    assert r["walk_mismatch"] == 0, r
    assert r["retained_overwritten"] == 0, r
    assert r["early_overwrite"] == 0, r
    windows = k >= 2 and k * W >= W + 64
    if windows or cap == 0:
        # windows: states 0, k, 2k, ...; a plain ring holding the whole
        # trajectory keeps every state (reported: the multiples of k)
        assert r["retained_states"] == T // k + 1
    else:  # a capped plain ring: the last cap + 1
        assert r["retained_states"] == cap + 1


# the paired-halves W = 16 kernel (pipe.hip PAIR): the default for
# W = 16 sweeps and long trajectories -- the 1024^2 x 500 trajectory and the
# 9-mu sweep's K = 4500 steps, short runs, and capped rings that wrap inside
# the launch
PAIRED = [(16, 500, 1, 0), (16, 4500, 1, 0), (16, 13, 1, 0), (16, 3, 1, 0), (16, 40, 1, 5),
          (16, 120, 1, 7), (16, 2, 1, 0)]


@pytest.mark.parametrize("W,T,k,cap", PAIRED)
def test_paired_walk_in_range_and_consistent(W, T, k, cap):
    r = _lib.ring_audit(W, T, k, cap, paired=True)
    assert r["accesses"] >= 2 * 8 * T * 64, r  # two cells per lane and paired diagonal
    assert r["out_of_range"] == 0, r
    assert 0 <= r["max_entry"] < r["entries_per_tile"], r
    assert r["walk_mismatch"] == 0, r  # per-diagonal walk = steady blocks = ring_pos
    assert r["retained_overwritten"] == 0, r
    assert r["early_overwrite"] == 0, r
    # the paired kernel keeps the same states as the one-cell kernel
    assert r["retained_states"] == _lib.ring_audit(W, T, k, cap)["retained_states"]


def test_paired_audit_catches_a_wrong_walk():
    """The paired replay is not vacuous: the one-cell walk's report differs
    from the paired one (different accesses), and the paired mode refuses
    widths and layouts the kernel never runs."""
    a = _lib.ring_audit(16, 13, 1, 0)
    b = _lib.ring_audit(16, 13, 1, 0, paired=True)
    assert a["accesses"] != b["accesses"]
    for bad in ((32, 13, 1, 0), (16, 13, 5, 0)):
        with pytest.raises(_lib.BurgersError):
            _lib.ring_audit(*bad, paired=True)


def test_ring_audit_rejects_bad_arguments():
    with pytest.raises(_lib.BurgersError):
        _lib.ring_audit(48, 10, 1, 0)  # not a pipe width
    with pytest.raises(_lib.BurgersError):
        _lib.ring_audit(64, 0, 1, 0)


def test_build_id_matches_checkout():
    """The library in the tree was built from the sources in the tree
    (burg_build_id vs the digest of csrc/ + Makefile + include/burgers.h)."""
    assert _lib.build_id() == _lib.source_id()


# the paired kernel's store wave in burg_sweep launches writes the paired
# sweep layout (ring_pos_paired: each half of a paired diagonal one
# contiguous entry): every cell's entry in range,
# equal to the extraction's mapping, and still holding its cell at the end
@pytest.mark.parametrize("T", [3, 13, 500, 4500])
def test_paired_sweep_layout_in_range_and_consistent(T):
    r = _lib.ring_audit(16, T, 1, 0, paired=True, paired_layout=True)
    assert r["accesses"] >= 2 * 8 * T * 64, r
    assert r["out_of_range"] == 0 and r["walk_mismatch"] == 0, r
    assert r["retained_overwritten"] == 0, r
    assert r["retained_states"] == T, r
    assert r["max_entry"] < r["entries_per_tile"], r


def test_paired_sweep_layout_needs_the_paired_walk():
    with pytest.raises(_lib.BurgersError):
        _lib.ring_audit(16, 13, 1, 0, paired=False, paired_layout=True)
    with pytest.raises(_lib.BurgersError):
        _lib.ring_audit(16, 13, 2, 0, paired=True, paired_layout=True)
