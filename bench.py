#!/usr/bin/env python3
"""Benchmark: Mcell-updates/s of the 2D inviscid Burgers FOM time loop.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--time-steps T]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Unit of work ("step"): ONE FOM TRAJECTORY = run_fom.main's time loop
(inviscid_burgers_implicit2D, C/hypernet2D.py:72-131): T = 500 implicit time
steps of the whole grid from w0 = 1 at mu = (5.19, 0.026), solved exactly by
the HIP march in ONE pipelined launch (burg_trajectory_ex), the snapshot
matrix kept resident in HBM (engine ring layout): every state when the whole
trajectory fits (N = 1, 4096^2: 134 GB), else every 10th state (--snap-every;
the N > 1 slabs: 268 / 537 GB would be needed per GPU) -- config.snap_every /
retained_states say which.
--sweep N times the snapshot sweep over the first N training mu instead
(burg_sweep; C/run_prom.py:59-71).

Workload, by GPU count (defaults; --nx / --rows-per-gpu override):
  N = 1: BASELINE.json configs[2] (the largest single-GPU config), 4096^2;
  N = 2: 8192 x 4096 (8192 x 2048 per GPU: configs[3]'s slab, half its rows);
  N = 4: BASELINE configs[3], 8192^2 (8192 x 2048 per GPU);
  N = 8: BASELINE configs[4], 16384^2 (16384 x 2048 per GPU: SURVEY.md 8(d)'s
         weak-scaling slab).
fp64, dt = 0.05 * 1024 / nx: the CFL number of the 1024^2 configuration
(dt = 0.05 there, as run_fom.py).  With dt = 0.05 at 4096^2 the reference
scheme itself is unstable (dt > 2h: v < 0 at the boundary, NaN after 14 steps
-- measured with the oracle), so a fixed dt would time
NaN arithmetic.  N > 1: row slabs, rank k owning rows [k*rows, (k+1)*rows) of
the nx x N*rows grid, the one-way halo streamed GPU-to-GPU during the launch
(DESIGN.md section 7).  value = nx * N*rows * T * K / (max over ranks of the
wall time of the K timed trajectories), inputs resident in HBM.
After the timed region every run checks its own result (residual_check):
the last step of a trajectory must solve the reference residual,
||R(w_T; w_{T-1})|| / ||R(w_{T-1}; w_{T-1})|| < 1e-13 (C/hypernet2D.py:2512-2570),
computed slab by slab with the south halo rows sent by the rank below
(burg_slab_residual + torch.distributed send/recv); the bench exits non-zero
if it fails.

Extra JSON objects: roofline (the march kernel: algorithmic 32 B per
cell-update = read the previous state u, v + write the new state u, v,
SURVEY.md section 8(d); per-launch device time from HIP events on the
library's stream; peak 8 TB/s; traffic from the committed rocprofv3 PMC
passes, profiles/pmc_traffic.json), issue_roofline (the compute waves'
instruction-issue floor per diagonal from the kernel ISA, tools/isa_count.py,
against the measured time per diagonal), cpu_baseline (the oracle's CPU
restatement, rank 0 at N = 1, bounded sample: the march on every host
thread, and the reference's Newton on one core), config2_1024 (BASELINE
configs[1]: the 1024^2 9-mu snapshot sweep) and end_to_end (run_fom.main's
timed region at 1024^2 x 500: march + D2H + .npy file).  Only the cpu_baseline leg
touches oracle/.  rom_pipeline: secondary numbers of the reference's ROM
driver at 250^2 (sweep, POD, LSPG; --no-rom skips).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
BYTES_PER_CELL_UPDATE = 32  # read up, vp + write u, v
MU = (5.19, 0.026)
DT = 0.05
METRIC = "Mcell-updates/s (fp64) for 2D Burgers FOM; % HBM roofline at 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10, help="timed sweeps")
    ap.add_argument("--warmup", type=int, default=2, help="untimed sweeps")
    ap.add_argument("--sweep", type=int, default=1,
                    help="trajectories per step: the first N of the 9 training mu "
                         "(get_snapshot_params); 1 = one trajectory at mu=(5.19, 0.026)")
    ap.add_argument("--time-steps", type=int, default=500,
                    help="implicit steps per trajectory (run_fom.py: 500)")
    ap.add_argument("--snap-every", type=int, default=0,
                    help="states kept in HBM per trajectory: every k-th (burg_trajectory_ex); "
                         "0 = auto: every state when the whole trajectory fits in HBM (4096^2: "
                         "134 GB), else every 10th (the 8192 x 2048 / 16384 x 2048 slabs)")
    ap.add_argument("--no-alone", action="store_true",
                    help="N > 1: skip per_gpu_alone (the per-GPU shape run as one rank first)")
    ap.add_argument("--nx", type=int, default=None,
                    help="row length (default by GPU count: 4096, 8192, 8192, 16384 for N = 1, 2, "
                         "4, 8)")
    ap.add_argument("--dt", type=float, default=None,
                    help="time step (default 0.05 * 1024 / nx: the 1024^2 config's CFL)")
    ap.add_argument("--no-1024", action="store_true",
                    help="skip the secondary BASELINE configs[1] line (1024^2 9-mu sweep)")
    ap.add_argument("--rows-per-gpu", type=int, default=None,
                    help="rows per GPU (default: nx at N = 1, 2048 at N > 1)")
    ap.add_argument("--no-residual-check", action="store_true",
                    help="skip the post-run residual check of the last step")
    ap.add_argument("--engine", default="pipe", choices=["pipe", "stream"])
    ap.add_argument("--stream-w", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-rom", action="store_true",
                    help="skip the secondary ROM-pipeline numbers (sweep, POD, LSPG at 250^2)")
    ap.add_argument("--stencil-nx", type=int, default=8192,
                    help="grid of the residual / J.x roofline probe (0: skip)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N > 1 rehearsal on a one-GPU box: every rank on device 0, gloo "
                         "for the host-side collectives (use small slabs so all ranks' "
                         "workgroups are resident together)")
    ap.add_argument("--pmc-file", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--isa-file", default=os.path.join(ROOT, "profiles", "r06", "pipe_isa.json"))
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end field (1024^2 x 500 trajectory + .npy file)")
    return ap.parse_args()


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, world, local


def host_threads():
    """CPU threads this process may use: the affinity mask, capped by
    OMP_NUM_THREADS when set (the GPU box sets it to its CPU share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


# BASELINE.json configs by (nx, ny, GPUs)
BASELINE_CONFIGS = {(1024, 1024, 1): 1, (4096, 4096, 1): 2, (8192, 8192, 4): 3,
                    (16384, 16384, 8): 4}
DEFAULT_SHAPES = {1: (4096, 4096), 2: (8192, 2048), 4: (8192, 2048), 8: (16384, 2048)}


def default_shape(world, nx=None, rows=None):
    """(nx, rows per GPU) of the bench by GPU count (module docstring)."""
    dnx, drows = DEFAULT_SHAPES.get(world, (8192, 2048))
    if nx is None:
        nx = dnx
        rows = rows or drows
    else:
        rows = rows or (nx if world == 1 else 2048)
    return nx, rows


def workload_label(nx, ny, world):
    k = BASELINE_CONFIGS.get((nx, ny, world))
    return f"BASELINE configs[{k}]" if k is not None else "not a BASELINE config"


def cpu_baseline(nx, dt, seconds):
    """The fastest CPU algorithm of this build on the bench's grid: the
    oracle's closed-form march (orc_march_sweep, the same arithmetic as the GPU
    kernel), one trajectory per host thread (the training mu of
    get_snapshot_params, cycled), OpenMP; steps sized so the sample takes about
    `seconds`.  Beside it, the reference algorithm itself (newton_raphson +
    exact block solve, C/hypernet2D.py:72-131,1811-1857) on one core."""
    from oracle import oracle
    from finitedifference_amd.config import get_snapshot_params
    P = oracle.Problem(nx, dt=dt)
    w0 = np.ones(P.m)
    thr = host_threads()
    mus = [get_snapshot_params()[j % 9] for j in range(thr)]
    t0 = time.perf_counter()
    P.march_sweep(w0, mus[:1], 1, 1)  # one step, one thread: sizes the sample
    t1 = time.perf_counter() - t0
    steps = max(1, int(seconds / max(t1, 1e-3) / 1.5))
    t0 = time.perf_counter()
    used = P.march_sweep(w0, mus, steps, thr)
    el = time.perf_counter() - t0
    march = nx * nx * steps * len(mus) / el / 1e6
    # the reference algorithm, one core, a short sample
    w = w0
    t0 = time.perf_counter()
    nsteps = 0
    while True:
        w, its, rel = P.newton_step(w)
        nsteps += 1
        if time.perf_counter() - t0 >= min(seconds, 6.0):
            break
    eln = time.perf_counter() - t0
    return {"value": round(march, 3), "unit": "Mcell-updates/s", "cores": int(used),
            "kind": "port", "nproc": os.cpu_count(),
            "threads_note": ("threads = this process's CPU share: the GPU pool gives a one-GPU "
                             "box 16 host threads (OMP_NUM_THREADS=16, affinity capped), while "
                             "nproc counts the whole machine"),
            "reference_measured": {
                "what": "the reference itself (C/run_fom.py -> inviscid_burgers_implicit2D, "
                        "NumPy/SciPy SuperLU, 1 core); it cannot run on the GPU box and is "
                        "infeasible at this grid (SuperLU: 183 s for ONE step at 1024^2, OOM "
                        "at 4096^2)",
                "coarse_250": {"value": 0.0501, "unit": "Mcell-updates/s", "cores": 1,
                               "source": "SURVEY.md section 6 / 8(d): 250^2 x 500 steps in "
                                         "623.3 s, build container (Xeon, "
                                         "OPENBLAS_NUM_THREADS=1)"},
                "fine_750_sherlock": {"value": 0.0116, "unit": "Mcell-updates/s", "cores": 1,
                                      "source": "F/output_55034725.log:1005 (the author's "
                                                "750^2 x 500 run on Sherlock), BASELINE.md"}},
            "sample": f"oracle march (orc_march_sweep, OpenMP) on {nx}x{nx}, dt={dt:g}: {len(mus)} "
                      f"trajectories (training mu) x {steps} steps from w0=1, one per thread, "
                      f"{el:.1f} s on {used} threads",
            "newton_1core": {"value": round(nx * nx * nsteps / eln / 1e6, 3),
                             "unit": "Mcell-updates/s", "cores": 1,
                             "sample": f"oracle Newton (reference algorithm, exact block solve in "
                                       f"place of SuperLU), first {nsteps} of the 500 steps, "
                                       f"{eln:.1f} s"}}


def end_to_end(nx=1024, T=500):
    """C/run_fom.py:41-43's timed region on the GPU: one {nx}^2 x {T}
    trajectory from w0 = 1 (dt = 0.05, mu = (5.19, 0.026)) including the
    snapshot matrix's device-to-host copy and its .npy file (burg_run_npy:
    pinned buffers, pwrite writer thread, no fsync as np.save), wall clock of the call; the file goes to
    a temporary directory and is deleted."""
    import tempfile
    from finitedifference_amd.solver import FOMContext
    ctx = FOMContext(nx, nx, engine="pipe")
    g = np.linspace(0, 100, nx + 1)
    ctx.set_problem(g, g, DT, MU)
    d = tempfile.mkdtemp(prefix="burg_e2e_")
    path = os.path.join(d, "snaps.npy")
    try:
        t0 = time.perf_counter()
        st = ctx.run_to_npy(np.ones(ctx.m), T, path)
        wall = time.perf_counter() - t0
        size = os.path.getsize(path)
        hdr = np.load(path, mmap_mode="r").shape
    except OSError as e:
        return {"error": f"{type(e).__name__}: {e}"}
    finally:
        ctx.close()
        if os.path.exists(path):
            os.remove(path)
        os.rmdir(d)
    return {"grid": f"{nx}x{nx}", "time_steps": T, "wall_s": round(wall, 3),
            "value": round(nx * nx * T / wall / 1e6, 3), "unit": "Mcell-updates/s",
            "march_kernel_ms": round(st["loop_ms"], 3), "file_bytes": size, "npy_shape": list(hdr),
            "what": "run_fom.main's timed region: march + D2H + np.save of the (2n, T+1) snapshot "
                    "matrix (burg_run_npy)"}


def block_of(W):
    """Diagonals per readiness block of the pipe kernel (pipe.hip uw_of):
    16 for wide tiles of 128 ... 1024 columns (512, 1024 since round 4),
    8 otherwise."""
    return 16 if W >= 128 else 8


def issue_roofline(kname, avg_ms, diagonals, isa_file, W, U=8, clock_ghz=None, clock_src=None):
    """Issue bound of the march kernel's compute waves: instructions per
    diagonal from the kernel's ISA (tools/isa_count.py -> profiles/r02/
    pipe_isa.json) at 4 cycles each (+12 per fp64 transcendental: one wave
    per SIMD issues at most one instruction per 4 cycles, tools/probes/
    issue_probe.hip), against the measured time per diagonal of the
    wavefront (its T*W diagonals plus its fill, nx + rows: the last tile
    starts that many diagonals after the first) at the kernel's effective
    clock (GRBM_GUI_ACTIVE in profiles/pmc_traffic.json; the nominal 2.4 GHz
    when absent).  Wide tiles mix interior and edge blocks ((64/U + 1) of
    every W/U blocks are edge blocks)."""
    if clock_ghz is None:
        clock_ghz, clock_src = 2.4, "nominal"
    try:
        d = json.load(open(isa_file))[kname]["per_diagonal_averages"]
    except Exception:
        return None
    if W <= 16 and "steady_edge_block" in d:
        # narrow tiles: all but ~1 % of the blocks (the first and last 64
        # diagonals, a sweep's trajectory starts) are steady-edge blocks
        cyc, ins = d["steady_edge_block"]["issue_cycles"], d["steady_edge_block"]["total"]
    elif "interior_block" in d:
        # interior blocks of full strips run the steady variant when built
        inner = d.get("steady_block", d["interior_block"])
        edge = d.get("steady_edge_block", d["edge_block"])
        fe = min(1.0, (64 / U + 1) / (W / U)) if W >= 128 else 1.0
        cyc = (1 - fe) * inner["issue_cycles"] + fe * edge["issue_cycles"]
        ins = (1 - fe) * inner["total"] + fe * edge["total"]
    else:
        cyc, ins = d["block"]["issue_cycles"], d["block"]["total"]
    meas = avg_ms * 1e6 / diagonals * clock_ghz
    return {"bound": "issue", "instructions_per_diagonal": round(ins, 1),
            "issue_cycles_per_diagonal": round(cyc, 1),
            "measured_cycles_per_diagonal": round(meas, 1), "frac": round(cyc / meas, 4),
            "clock_ghz": clock_ghz, "clock_source": clock_src, "wavefront_diagonals": diagonals,
            "source": os.path.relpath(isa_file, ROOT)}


def stencil_roofline(nx, reps=20, pmc_file=None):
    """Residual (K1) and Jacobian action (K2) -- the HBM-bound stencils of the
    reference's Newton path (C/hypernet2D.py:2512-2570, 2627-2656) -- on an
    nx x nx grid (north star: >= 40 % of HBM roofline at 8192^2).  Algorithmic
    bytes per launch: 48 B per cell; mean launch time
    from HIP events on the library's stream."""
    from finitedifference_amd.solver import FOMContext
    ctx = FOMContext(nx, nx, engine="pipe")
    g = np.linspace(0, 100, nx + 1)
    ctx.set_problem(g, g, DT, MU)
    rng = np.random.default_rng(1234557)
    ctx.upload(rng.uniform(1.0, 6.0, ctx.m))
    out = {"grid": f"{nx}x{nx}", "alg_bytes_per_cell": 48, "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    for k in ("residual", "jvp"):
        ms = ctx.kernel_bench(k, reps)
        gbs = 48.0 * nx * nx / (ms * 1e-3) / 1e9
        traffic, tsrc = read_pmc(pmc_file, f"stencil_{k}:{nx}x{nx}") if pmc_file else (None, None)
        out[k] = {"avg_launch_ms": round(ms, 5), "achieved": round(gbs, 1),
                  "frac": round(gbs / HBM_PEAK_GBS, 4), "alg_bytes": 48 * nx * nx,
                  "traffic": traffic, "traffic_source": tsrc}
    ctx.close()
    return out


ROM_MUS = [(4.25, 0.015), (4.25, 0.0225), (4.25, 0.03), (4.875, 0.015), (4.875, 0.0225),
           (4.875, 0.03), (5.5, 0.015), (5.5, 0.0225), (5.5, 0.03)]


def rom_pipeline(N=250, T=500, npod=95, rom_steps=20):
    """The reference's ROM driver (C/run_prom.py:24-110) on the GPU at its own
    size (250^2, 9 training mu x 500 steps, 95 POD modes): the FOM snapshot
    sweep, POD (rsvd), and LSPG PROM steps at the out-of-sample mu
    (4.75, 0.02).  Secondary numbers -- not the headline metric.  The LSPG
    fused J.basis + Gram kernel's achieved rate is on its algorithmic bytes
    (DESIGN.md section 4.6)."""
    from finitedifference_amd import hypernet2D as H
    from finitedifference_amd.solver import FOMContext
    import torch
    gx, gy = H.make_2D_grid(0, 100, 0, 100, N, N)
    m = 2 * N * N
    H.inviscid_burgers_implicit2D_sweep(gx, gy, np.ones(m), DT, 2, ROM_MUS, verbose=0)  # warm
    t0 = time.perf_counter()
    sn, sst = H.inviscid_burgers_implicit2D_sweep(gx, gy, np.ones(m), DT, T, ROM_MUS, verbose=0,
                                                  return_stats=True)
    t_sweep = time.perf_counter() - t0
    S = np.hstack(sn)
    del sn
    # warm-up on a slice: loads the rocBLAS / rocSOLVER code objects, which the
    # first call in a process otherwise pays inside its timed region
    H.POD(np.ascontiguousarray(S[:, :256]), num_modes=npod, method="rsvd", random_state=0)
    u, s, pod_ms = H.POD(S, num_modes=npod, method="rsvd", random_state=0, return_ms=True)
    del S
    # the same flow with the snapshot set left on the device (burg_sweep_device
    # -> burg_pod_rsvd_device): no 4.5 GB host round trip
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Sd, dst = H.inviscid_burgers_implicit2D_sweep(gx, gy, np.ones(m), DT, T, ROM_MUS, verbose=0,
                                                  on_device=True, return_stats=True)
    ud, sd, pod_ms_dev = H.POD(Sd, num_modes=npod, method="rsvd", random_state=0, return_ms=True)
    t_dev = time.perf_counter() - t0
    del Sd
    torch.cuda.empty_cache()
    pod_match = float(np.max(np.abs(sd - s) / s[0]))
    ctx = FOMContext(N, N)
    ctx.set_problem(gx, gy, DT, (4.75, 0.02))
    ctx.lspg(np.ones(m), 1, u, keep_snaps=False)  # warm-up
    _, _, its, _, times, st = ctx.lspg(np.ones(m), rom_steps, u, keep_snaps=False)
    ctx.close()
    upd = max(st["newton_updates"], 1)
    gram_ms = times[0] / upd
    alg = 2 * m * npod * 8 + 4 * m * 8
    return {"grid": f"{N}x{N}", "training": f"{len(ROM_MUS)} mu x {T} steps", "npod": npod,
            "fom_sweep_s_incl_d2h": round(t_sweep, 3), "pod_rsvd_device_ms": round(pod_ms, 2),
            "fom_sweep_kernel_ms": round(sst["loop_ms"], 3),
            "fom_sweep_launches": sst["stream_launches"],
            "fom_sweep_tile_w": sst["stream_w"],
            "fom_sweep_gcell_per_s": round(m // 2 * T * len(ROM_MUS) / sst["loop_ms"] / 1e6, 2),
            "sweep_to_pod_on_device_s": round(t_dev, 3),
            "sweep_to_pod_on_device_detail": {
                "sweep_kernel_ms": round(dst["loop_ms"], 3), "pod_ms": round(pod_ms_dev, 2),
                "what": "burg_sweep_device (the 9 trajectories side by side, snapshot set left "
                        "in HBM) + burg_pod_rsvd_device, wall clock",
                "sigma_max_rel_diff_vs_host_path": pod_match},
            "lspg_ms_per_step": round(st["loop_ms"] / rom_steps, 4),
            "lspg_gn_norms_per_step": float(its.mean()),
            "lspg_gram": {"avg_launch_ms": round(gram_ms, 4), "alg_bytes": alg,
                          "achieved": round(alg / gram_ms / 1e6, 1), "unit": "GB/s",
                          "frac": round(alg / gram_ms / 1e6 / HBM_PEAK_GBS, 4)},
            "reference_cpu_1core_build_container": {
                "lspg_s_per_step": 1.03, "pod_rsvd_s": 49.6,
                "source": "profiles/r01/lspg/reference_cpu_timing.txt, "
                          "profiles/r01/pod/reference_cpu_timing.txt"}}


def read_pmc(path, key):
    try:
        d = json.load(open(path))
    except Exception:
        return None, None
    e = d.get(key)
    if not e:
        return None, None
    return e.get("hbm_bytes_per_launch"), e.get("source")


def read_clock(path, key):
    """(effective clock GHz, source) of a kernel from profiles/pmc_traffic.json."""
    try:
        e = json.load(open(path)).get(key) or {}
    except Exception:
        return None, None
    return e.get("effective_clock_ghz"), e.get("clock_source")


def _lib_build_id():
    from finitedifference_amd import _lib
    return _lib.build_id()


def _lib_source_id():
    from finitedifference_amd import _lib
    return _lib.source_id()


def _lib_build_flags():
    from finitedifference_amd import _lib
    return _lib.build_flags()


HALO_MODES = {0: None, 1: "pinned host memory", 2: "consumer GPU memory over IPC (xGMI)"}


def rank_diag(ctx, st, rank, kern_ms, launches, snap_every):
    """What one rank of an N > 1 line saw: its kernel
    time, the launch's ramp (first workgroup entry -> the last compute wave's
    first block) and the wait for the rank below (-> the halo strip's first
    block), south-inflow waits at the slab boundary (the halo ring) against
    the in-GPU strip boundaries, the halo placement of both boundaries and why
    a device ring was not used, the resolved snap_every, and the bounds-guard
    counters (DESIGN.md sections 6.1, 7)."""
    hin, hout = ctx.halo_modes()
    return {"rank": rank,
            "kernel_ms_last": round(st["loop_ms"], 3),
            "kernel_ms_avg": round(kern_ms / max(launches, 1), 3),
            "ramp_ms": round(st["ramp_ms"], 3),
            "halo_wait_ms": round(st["halo_wait_ms"], 3),
            "south_waits_halo": st["south_waits_halo"],
            "south_wait_ms_halo": round(st["south_wait_ms_halo"], 3),
            "south_waits_local": st["south_waits_local"],
            "south_wait_ms_local": round(st["south_wait_ms_local"], 3),
            "halo_in": HALO_MODES[hin], "halo_out": HALO_MODES[hout],
            "halo_note": ctx.halo_note(),
            "snap_every": snap_every,
            "bounds_guard": {"checks": st["bounds_checks"], "hits": st["bounds_hits"]}}


def main():
    args = parse()
    rank, world, local = dist_env()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (use torchrun for N > 1)",
              file=sys.stderr)
        sys.exit(2)
    nx, rows = default_shape(world, args.nx, args.rows_per_gpu)
    ny = rows * world
    T = args.time_steps
    dt = args.dt if args.dt is not None else DT * 1024.0 / nx
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

    import torch
    import torch.distributed as dist
    from finitedifference_amd.dist import make_slab_context

    rehearse = world > 1 and args.rehearse_one_gpu
    dev = 0 if rehearse else local
    if world > 1:
        torch.cuda.set_device(dev)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from finitedifference_amd.config import get_snapshot_params
    mus = get_snapshot_params()[:args.sweep] if args.sweep > 1 else [MU]
    nmu = len(mus)
    gx = np.linspace(0, 100, nx + 1)
    gy = np.linspace(0, 100.0 * ny / nx, ny + 1)  # same cell size: weak scaling

    def setup():
        c = make_slab_context(nx, ny, rank, world, device=dev if world > 1 else 0,
                              dist=dist if world > 1 else None, engine=args.engine,
                              stream_w=args.stream_w)
        c.set_problem(gx, gy, dt, MU, allow_nonsquare=(nx != ny))
        c.upload(np.ones(c.m))
        if nmu == 1:
            if world > 1 and args.snap_every <= 0:
                # "auto" resolves per rank from its own free HBM: agree on the
                # largest stride, so every rank keeps the same states
                k, _, _ = c.trajectory_plan(T, args.snap_every)
                t = torch.tensor([k], dtype=torch.int64, device="cpu" if rehearse else "cuda")
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                args.snap_every = int(t.item())
            # the trajectory ring (134 GB at 4096^2 x 500 steps) is allocated
            # here, before the barrier: no rank's first launch waits on a
            # neighbour still allocating (the halo waits are bounded in time)
            c.reserve(T, snap_every=args.snap_every)
        return c

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def measure(c):
        """Warm-up and timed trajectories.  Every rank runs the same sequence
        of collectives whatever happens: a step that raises records the error
        and the rank skips its remaining launches (its neighbours' bounded halo
        waits then give up too), so the agreement below always pairs up."""
        err = []

        def one_step():
            if err:
                return None
            try:
                if nmu == 1:
                    return c.trajectory(T, snap_every=args.snap_every)
                return c.sweep(mus, T, keep_snaps=False)[1]
            except BurgersError as e:
                err.append(e)
                return None
        for _ in range(args.warmup):
            barrier()
            one_step()
        barrier()
        t0 = time.perf_counter()
        kern = 0.0
        nl = 0
        s = None
        for _ in range(args.steps):
            s = one_step()
            if s is not None:
                kern += s["loop_ms"]
                nl += max(1, s["stream_launches"])
        barrier()
        return (time.perf_counter() - t0, kern, nl, s), (err[0] if err else None)

    def agree(c, e):
        """0: every rank ok; 1: some rank's device halo ring stalled (a wait
        timed out with a device ring on one of its boundaries) -- fall back to
        the host rings; 2: any other failure -- re-raise everywhere."""
        code = 0
        if e is not None:
            hin, hout = c.halo_modes()
            code = 1 if ("wait timed out" in str(e) and 2 in (hin, hout)) else 2
        if world == 1:
            return code
        t = torch.tensor([code], dtype=torch.int32, device="cpu" if rehearse else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.item())

    from finitedifference_amd._lib import BurgersError
    alone = None
    if world > 1 and nmu == 1 and not args.no_alone:
        # the same per-GPU shape as ONE rank (no halo) on rank 0's GPU, before
        # the collective run: the weak-scaling reference that separates the
        # halo / ramp cost from the tile shape's own rate
        if rank == 0:
            alone = per_gpu_alone(nx, rows, dt, T, args, dev)
        dist.barrier()
    ctx = setup()
    halo_fallback = None
    res, err = measure(ctx)
    code = agree(ctx, err)
    if code == 1 and os.environ.get("BURG_HALO") != "host":
        halo_fallback = f"device halo ring failed ({err or 'on another rank'}); host rings"
        print(f"bench.py rank {rank}: {halo_fallback}", file=sys.stderr, flush=True)
        ctx.close()
        os.environ["BURG_HALO"] = "host"
        os.environ.pop("BURG_TEST_FAIL_DEVICE_HALO", None)
        ctx = setup()
        res, err = measure(ctx)
        code = agree(ctx, err)
    if code:
        raise RuntimeError(f"rank {rank}: the timed run failed ({err or 'on another rank'})")
    elapsed, kern_ms, launches, st = res
    # what the timed trajectories kept resident (before the residual check reuses the ring)
    ret_first, ret_count, ret_stride = ctx.retained() if nmu == 1 else (0, 0, 0)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearse else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    check = None
    if not args.no_residual_check:
        check = residual_check(ctx, T, dist if world > 1 else None,
                               None if rehearse or world == 1 else dev, args.snap_every)
    cells = nx * ny  # whole job
    value = cells * T * nmu * args.steps / elapsed / 1e6

    st_main = st
    halo = None
    per_rank = None
    if world > 1:
        hin, hout = ctx.halo_modes()
        halo = HALO_MODES[hout if rank == 0 else hin]
        note = ctx.halo_note()
        if note:
            halo += f" ({note})"
        per_rank = [None] * world
        dist.all_gather_object(per_rank, rank_diag(ctx, st, rank, kern_ms, launches, ret_stride))
    ctx.close()  # give the trajectory ring back before the secondary probes
    if rank == 0:
        st = st_main
        eng = {0: "stream", 2: "pipe"}.get(st["engine"], str(st["engine"]))
        kname = (f"pipe_kernel<{st['stream_w']}, {'true' if nmu > 1 else 'false'}>"
                 if st["engine"] == 2 else f"stream_kernel<{st['stream_w']}>")
        # this rank's kernel: all launches of the timed region
        per_launch = BYTES_PER_CELL_UPDATE * nx * rows * T * nmu * args.steps / launches
        avg_ms = kern_ms / launches
        achieved = per_launch / (avg_ms * 1e-3) / 1e9
        key = f"{eng}:{nx}x{rows}:T{T}" + (f"x{nmu}" if nmu > 1 else "")
        traffic, tsrc = read_pmc(args.pmc_file, key)
        what = (f"the FOM snapshot sweep over the first {nmu} training mu of get_snapshot_params "
                f"(C/train_autoencoder.py:63-72, as run_prom.py:59-71), {T} steps each"
                if nmu > 1 else
                f"one {T}-step FOM trajectory from w0 at mu=(5.19,0.026) (run_fom.main's loop)")
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mcell-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": (f"synthetic: reference initial state w0=1, dt={dt:g} (0.05*1024/nx: the "
                     f"1024^2 config's CFL), domain cell size 100/{nx}; each step = {what}"),
            "config": {
                "workload": f"implicit 2D inviscid Burgers FOM (run_fom time loop), "
                            f"{nx}x{rows} cells per GPU (grid {nx}x{ny}), fp64, "
                            f"{T} implicit steps per trajectory, {nmu} trajectories (mu) "
                            f"per step, exact march on {world}x MI355X "
                            f"({workload_label(nx, ny, world)})",
                "baseline_config": BASELINE_CONFIGS.get((nx, ny, world)),
                "nx": nx, "ny": ny, "rows_per_gpu": rows, "time_steps": T, "dt": dt,
                "trajectories_per_step": nmu,
                "snap_every": ret_stride if nmu == 1 else None,
                "retained_states": ret_count if nmu == 1 else None,
                "retained_first_state": ret_first if nmu == 1 else None,
                "retained_note": ("states kept in HBM per trajectory and GPU (burg_trajectory_ex): "
                                  "every state while the whole trajectory fits, else every "
                                  "snap_every-th in retained ring windows (no extra traffic); "
                                  "the reference keeps every state in host memory"
                                  if nmu == 1 else None),
                "parallelism": f"row-slab x{world}",
                "halo_ring": halo,
                "halo_fallback": halo_fallback,
            },
            "residual_check": check,
            "build_id": {"library": _lib_build_id(), "sources": _lib_source_id(),
                         "flags": _lib_build_flags()},
            "engine": {"name": eng, "tile_w": st["stream_w"], "tiles": st["stream_tiles"],
                       "blocked_diagonals": st["slow_diagonals"],
                       "spin_polls": st["stall_spins"], "ieee_diagonals": st["ieee_diagonals"],
                       "comm_polls": st["comm_polls"], "ramp_ms": round(st["ramp_ms"], 3),
                       "bounds_guard": {"checks": st["bounds_checks"], "hits": st["bounds_hits"],
                                        "what": "copy calls of this context that checked the "
                                                "ring/transpose kernels' bounds guard (err[5], "
                                                "DESIGN.md section 6.1), and hits (each one "
                                                "fails its call)"}},
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "kernel": kname,
                "per_launch_alg_bytes": int(per_launch),
                "avg_launch_ms": round(avg_ms, 5),
                "launches": launches,
                "traffic_source": tsrc,
            },
        }
        if per_rank is not None:
            out["per_rank"] = per_rank
        if alone is not None:
            out["per_gpu_alone"] = alone
            out["weak_eff_same_shape"] = round(value / (world * alone["value"]), 4)
        if st["engine"] == 2:
            clk, csrc = read_clock(args.pmc_file, key)
            iss = issue_roofline(kname, avg_ms, T * nmu * st["stream_w"] + nx + rows,
                                 args.isa_file, st["stream_w"], U=block_of(st["stream_w"]),
                                 clock_ghz=clk, clock_src=csrc)
            if iss:
                out["issue_roofline"] = iss
        if world == 1 and not args.no_1024:
            out["config2_1024"] = config2_1024(args.pmc_file, args.isa_file)
            out["single_1024"] = single_1024(args.pmc_file, args.isa_file)
        if world == 1 and not args.no_e2e:
            out["end_to_end"] = end_to_end()
        if world == 1 and args.stencil_nx > 0:
            out["stencil_roofline"] = stencil_roofline(args.stencil_nx, pmc_file=args.pmc_file)
        if world == 1 and not args.no_rom:
            out["rom_pipeline"] = rom_pipeline()
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(nx, dt, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if check is not None and not check["ok"]:
        print(f"bench.py: residual check failed: {check}", file=sys.stderr, flush=True)
        sys.exit(3)


def per_gpu_alone(nx, rows, dt, T, args, dev):
    """One rank's shape (nx x rows cells, the slab's cell size and dt) as a
    single-domain context on `dev`: W untimed + min(K, 3) timed trajectories,
    the same snap_every; Mcell-updates/s of one GPU with no halo."""
    import torch
    from finitedifference_amd.solver import FOMContext
    c = FOMContext(nx, rows, device=dev, engine=args.engine, stream_w=args.stream_w)
    c.set_problem(np.linspace(0, 100, nx + 1), np.linspace(0, 100.0 * rows / nx, rows + 1), dt, MU,
                  allow_nonsquare=(nx != rows))
    c.upload(np.ones(c.m))
    c.reserve(T, snap_every=args.snap_every)
    for _ in range(max(1, args.warmup)):
        c.trajectory(T, snap_every=args.snap_every)
    k = max(1, min(args.steps, 3))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kern = 0.0
    for _ in range(k):
        kern += c.trajectory(T, snap_every=args.snap_every)["loop_ms"]
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    f, n, stride = c.retained()
    c.close()
    return {"value": round(nx * rows * T * k / el / 1e6, 3), "unit": "Mcell-updates/s",
            "shape": f"{nx}x{rows}", "trajectories": k,
            "kernel_ms": round(kern / k, 3), "snap_every": stride, "retained_states": n,
            "what": "the per-GPU shape of this line run as ONE rank (single domain, no halo) on "
                    "rank 0's GPU before the collective run; weak_eff_same_shape = value / "
                    "(n_gpus * this)"}


RESIDUAL_TOL = 1e-13


def residual_check(ctx, T, dist=None, device=None, snap_every=1):
    """The run checks its own result: w_{T-1} and w_T of the bench's
    trajectory (burg_trajectory from w0 at mu = (5.19, 0.026)) are taken from
    two more launches, and the last step must solve the reference residual
    (C/hypernet2D.py:2512-2570): ||R(w_T; w_{T-1})|| / ||R(w_{T-1}; w_{T-1})||
    < RESIDUAL_TOL, norms over the whole grid (slab residuals with the halo
    rows from the rank below, summed over ranks).  Also the largest per-slab
    ratio (max over ranks)."""
    from finitedifference_amd.dist import slab_residual_norms
    if T >= 2:
        ctx.trajectory(T - 1, snap_every=snap_every)
        wpm = ctx.download()
    else:
        wpm = np.ones(ctx.m)  # the uploaded w0
    ctx.trajectory(T, snap_every=snap_every)
    wT = ctx.download()
    n1, s1 = slab_residual_norms(ctx, wT, wpm, dist, device)
    n0, s0 = slab_residual_norms(ctx, wpm, wpm, dist, device)
    rel = n1 / n0 if n0 > 0 else float("inf")
    srel = s1 / s0 if s0 > 0 else float("inf")
    if dist is not None:
        import torch
        t = torch.tensor([srel], dtype=torch.float64,
                         device="cpu" if device is None else torch.device("cuda", device))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        srel = float(t.item())
    return {"what": "||R(w_T; w_(T-1))|| / ||R(w_(T-1); w_(T-1))|| of the last step, reference "
                    "residual res2D_alt (C/hypernet2D.py:2512-2570), slab by slab with the halo "
                    "rows from the rank below",
            "rel": rel, "max_over_ranks_slab_rel": srel, "norm_R_T": n1, "norm_R_T-1": n0,
            "tol": RESIDUAL_TOL, "ok": bool(rel < RESIDUAL_TOL and srel < RESIDUAL_TOL)}


def single_1024(pmc_file, isa_file=None, steps=5):
    """run_fom.main's own unit at BASELINE configs[1]: ONE 1024^2 x 500
    trajectory (dt = 0.05, mu = (5.19, 0.026), w0 = 1) in one burg_trajectory
    launch, every state kept in HBM -- priced against the HBM roofline (32 B
    per cell-update), against its PMC traffic and against the compute waves'
    issue floor; secondary to the headline."""
    from finitedifference_amd.solver import FOMContext
    nx, T = 1024, 500
    ctx = FOMContext(nx, nx, engine="pipe")
    g = np.linspace(0, 100, nx + 1)
    ctx.set_problem(g, g, DT, MU)
    ctx.upload(np.ones(ctx.m))
    ctx.reserve(T)
    ctx.trajectory(T)
    t0 = time.perf_counter()
    kern = 0.0
    for _ in range(steps):
        st = ctx.trajectory(T)
        kern += st["loop_ms"]
    el = time.perf_counter() - t0
    ctx.close()
    upd = nx * nx * T
    ms = kern / steps
    gbs = BYTES_PER_CELL_UPDATE * upd / (ms * 1e-3) / 1e9
    key = f"pipe:{nx}x{nx}:T{T}"
    traffic, tsrc = read_pmc(pmc_file, key)
    clk, csrc = read_clock(pmc_file, key)
    paired = st.get("paired_launches", 0) > 0
    W = st["stream_w"]
    if paired:
        kname = f"pipe_kernel<{W}, false, paired (per cell)>"
        cell_diags = 2 * (T * W // 2 + 2 * nx)
    else:
        kname = f"pipe_kernel<{W}, false>"
        cell_diags = T * W + 2 * nx
    iss = issue_roofline(kname, ms, cell_diags, isa_file, W, U=block_of(W), clock_ghz=clk,
                         clock_src=csrc) if isa_file else None
    meas = (round(traffic / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
            if isinstance(traffic, (int, float)) and traffic > 0 else None)
    return {"grid": f"{nx}x{nx}", "dt": DT, "unit_of_work": f"one trajectory x {T} steps "
                                                          "(run_fom.main's loop)",
            "value": round(upd * steps / el / 1e6, 3), "unit": "Mcell-updates/s",
            "kernel": kname, "tile_w": W, "tiles": st["stream_tiles"],
            "avg_launch_ms": round(ms, 4), "ramp_ms": round(st["ramp_ms"], 3),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 5),
                         "per_launch_alg_bytes": BYTES_PER_CELL_UPDATE * upd,
                         "traffic": traffic, "traffic_source": tsrc,
                         "frac_measured_traffic": meas},
            "issue_roofline": iss, "paired_halves": paired,
            "ieee_diagonals": st["ieee_diagonals"]}


def config2_1024(pmc_file, isa_file=None, steps=3):
    """BASELINE configs[1] (1024^2, dt = 0.05 as run_fom.py): the 9-mu FOM
    snapshot sweep in one burg_sweep launch (pipe_kernel<16, true>), every
    state kept in HBM; secondary to the headline."""
    from finitedifference_amd.config import get_snapshot_params
    from finitedifference_amd.solver import FOMContext
    nx, T = 1024, 500
    mus = get_snapshot_params()[:9]
    ctx = FOMContext(nx, nx, engine="pipe")
    g = np.linspace(0, 100, nx + 1)
    ctx.set_problem(g, g, DT, MU)
    ctx.upload(np.ones(ctx.m))
    ctx.sweep(mus, T, keep_snaps=False)
    t0 = time.perf_counter()
    kern = 0.0
    for _ in range(steps):
        st = ctx.sweep(mus, T, keep_snaps=False)[1]
        kern += st["loop_ms"]
    el = time.perf_counter() - t0
    ctx.close()
    upd = nx * nx * T * len(mus)
    ms = kern / steps
    gbs = BYTES_PER_CELL_UPDATE * upd / (ms * 1e-3) / 1e9
    traffic, tsrc = read_pmc(pmc_file, f"pipe:{nx}x{nx}:T{T}x9")
    paired = st.get("paired_launches", 0) > 0
    clk, csrc = read_clock(pmc_file, f"pipe:{nx}x{nx}:T{T}x9")
    if paired:
        # the paired-halves kernel: two cells per lane
        # and diagonal, T * nmu * 8 + 2 nx paired diagonals; the ISA counts
        # and the issue bound are per CELL, so the measured side is too
        kname = f"pipe_kernel<{st['stream_w']}, true, paired (per cell)>"
        cell_diags = 2 * (T * len(mus) * st["stream_w"] // 2 + 2 * nx)
    else:
        kname = f"pipe_kernel<{st['stream_w']}, true>"
        cell_diags = T * len(mus) * st["stream_w"] + 2 * nx
    iss = issue_roofline(kname, ms, cell_diags, isa_file, st["stream_w"],
                         U=block_of(st["stream_w"]), clock_ghz=clk,
                         clock_src=csrc) if isa_file else None
    # the narrow tiles keep the previous state in LDS: the bytes they move
    # (PMC) are ~0.6 x the 32-B model's, so the fraction on measured traffic
    # says how close to HBM they actually run
    meas = (round(traffic / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
            if isinstance(traffic, (int, float)) and traffic > 0 else None)
    return {"grid": f"{nx}x{nx}", "dt": DT, "unit_of_work": f"9-mu snapshot sweep x {T} steps",
            "issue_roofline": iss,
            "value": round(upd * steps / el / 1e6, 3), "unit": "Mcell-updates/s",
            "kernel": kname, "avg_launch_ms": round(ms, 4),
            "roofline_frac": round(gbs / HBM_PEAK_GBS, 5), "achieved_GBs": round(gbs, 1),
            "roofline_frac_measured_traffic": meas,
            "roofline_frac_note": "roofline_frac: 32 B per cell-update (SURVEY 8(d)) / kernel "
                                  "time / 8 TB/s; _measured_traffic: PMC HBM bytes per launch "
                                  "(traffic) / kernel time / 8 TB/s",
            "ieee_diagonals": st["ieee_diagonals"], "paired_halves": paired,
            "traffic": traffic, "traffic_source": tsrc}


if __name__ == "__main__":
    main()
