"""CPU: the committed N = 2 rehearsal line (two slab ranks sharing one GPU,
tools/gpu_r6.sh -> profiles/r06/) carries the per-rank diagnostics a
multi-GPU bench line must explain itself with: kernel
time, the ramp and the wait for the rank below, south-inflow waits at the
slab boundary against the in-GPU ones, both halo placements and the note,
the resolved snap_every, and the bounds-guard counters."""
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PER_RANK = ("rank", "kernel_ms_last", "kernel_ms_avg", "ramp_ms", "halo_wait_ms", "south_waits_halo",
            "south_wait_ms_halo", "south_waits_local", "south_wait_ms_local", "halo_in", "halo_out",
            "halo_note", "snap_every", "bounds_guard")


def _lines():
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r06", "*", "bench_rehearse_n2.json")))
    assert paths, "no committed N = 2 rehearsal line under profiles/r06/"
    return [(p, json.loads(open(p).read().strip().splitlines()[-1])) for p in paths]


def test_rehearsal_line_has_per_rank_diagnostics():
    for path, line in _lines():
        assert line["n_gpus"] == 2 and len(line["per_rank"]) == 2, path
        for r, d in enumerate(line["per_rank"]):
            assert tuple(d) == PER_RANK or set(PER_RANK) <= set(d), (path, d)
            assert d["rank"] == r
            assert d["kernel_ms_last"] > 0 and d["ramp_ms"] > 0
            assert d["bounds_guard"]["hits"] == 0
        r0, r1 = line["per_rank"]
        # rank 0 has no inbound halo; rank 1 reads the ring rank 0 writes
        assert r0["halo_in"] is None and r0["halo_wait_ms"] == -1 and r0["south_waits_halo"] == 0
        assert r1["halo_out"] is None and r1["halo_wait_ms"] >= 0
        assert r0["halo_out"] == r1["halo_in"] is not None
        assert r0["snap_every"] == r1["snap_every"] == line["config"]["snap_every"]


def test_bench_line_reports_bounds_guard_and_build_flags():
    for path, line in _lines():
        assert line["build_id"]["flags"].endswith("knobs: none"), path
        assert line["engine"]["bounds_guard"]["hits"] == 0
