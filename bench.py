#!/usr/bin/env python3
"""Benchmark: Mcell-updates/s of the 2D inviscid Burgers FOM time loop.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--nx 1024] [--rows-per-gpu R]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Workload (BASELINE.json configs[1]): 1024 x 1024 cells per GPU, fp64,
dt = 0.05, mu = (5.19, 0.026), w0 = 1 (the reference run_fom.py defaults,
C/run_fom.py:24-38), implicit step solved exactly by the HIP march.  A "step"
is one implicit time step of the whole grid.  N > 1: weak scaling by row
slabs (each rank owns R rows of an nx x (R*N) grid, same cell size, halo over
RCCL).  value = N * cells_per_rank * K / max-over-ranks wall time of the K
timed steps, inputs resident in HBM.

Extra JSON objects: roofline (march kernel, algorithmic 32 B/cell-update,
HIP-event kernel time, peak 8 TB/s) and cpu_baseline (the oracle's CPU
restatement of the reference Newton algorithm, rank 0 at N = 1, bounded
sample).  Only the cpu_baseline leg touches oracle/.
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nx", type=int, default=1024)
    ap.add_argument("--rows-per-gpu", type=int, default=None)
    ap.add_argument("--engine", default="stream", choices=["stream", "tiles"])
    ap.add_argument("--stream-w", type=int, default=0)
    ap.add_argument("--tiles-target", type=int, default=0)
    ap.add_argument("--tile-w", type=int, default=64)
    ap.add_argument("--tol", type=float, default=2.0 ** -50)
    ap.add_argument("--profile-steps", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-file", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, world, local


def cpu_baseline(nx, seconds):
    """Oracle restatement of the reference algorithm (newton_raphson + exact
    block solve, C/hypernet2D.py:72-131,1811-1857) on the host, 1 thread,
    first steps of the same 1024^2 trajectory until `seconds` elapse."""
    from oracle import oracle
    P = oracle.Problem(nx)
    w = np.ones(P.m)
    t0 = time.perf_counter()
    steps = 0
    while True:
        w, its, rel = P.newton_step(w)
        steps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": nx * nx * steps / dt / 1e6, "unit": "Mcell-updates/s", "cores": 1,
            "kind": "port",
            "sample": f"oracle Newton (reference algorithm, exact block solve in place of "
                      f"SuperLU) on {nx}x{nx}, first {steps} steps from w0=1, {dt:.1f} s, "
                      f"1 thread"}


def read_pmc(path, nx, ny):
    try:
        d = json.load(open(path))
    except Exception:
        return None, None
    key = f"{nx}x{ny}"
    e = d.get(key)
    if not e:
        return None, None
    return e.get("hbm_bytes_per_launch"), e.get("source")


def main():
    args = parse()
    rank, world, local = dist_env()
    if world != args.gpus:
        if args.gpus > 1 and world == 1:
            print(f"bench.py: --gpus {args.gpus} needs torchrun (one rank per GPU)",
                  file=sys.stderr)
            sys.exit(2)
    nx = args.nx
    rows = args.rows_per_gpu or nx
    ny = rows * world
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

    import torch
    import torch.distributed as dist
    from finitedifference_amd.dist import make_slab_context

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    ctx = make_slab_context(nx, ny, rank, world, device=local if world > 1 else 0,
                            tile_w=args.tile_w, tol=args.tol, engine=args.engine,
                            stream_w=args.stream_w, tiles_target=args.tiles_target)
    gx = np.linspace(0, 100, nx + 1)
    gy = np.linspace(0, 100.0 * ny / nx, ny + 1)  # same cell size: weak scaling
    ctx.set_problem(gx, gy, DT, MU, allow_nonsquare=(nx != ny))
    ctx.upload(np.ones(ctx.m))

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    if args.warmup > 0:
        ctx.advance(args.warmup)
    barrier()
    t0 = time.perf_counter()
    st = ctx.advance(args.steps)
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    cells = nx * ny  # whole job
    value = cells * args.steps / elapsed / 1e6

    # roofline leg: time every march launch with HIP events on the library stream
    prof = None
    if args.profile_steps > 0:
        ctx.set_options(tile_w=args.tile_w, tol=args.tol, profile=True)
        pst = ctx.advance(args.profile_steps)
        ctx.set_options(tile_w=args.tile_w, tol=args.tol, profile=False)
        if pst["march_launches"] > 0:
            alg_bytes = BYTES_PER_CELL_UPDATE * (nx * rows) * args.profile_steps
            launches = pst["march_launches"]
            avg_ms = pst["march_kernel_ms"] / launches
            per_launch = alg_bytes / launches
            achieved = per_launch / (avg_ms * 1e-3) / 1e9
            kname = (f"stream_kernel<{pst['stream_w']}>" if pst["engine"] == 0
                     else f"march_pass_kernel<{args.tile_w}>")
            prof = dict(launches=launches, avg_ms=avg_ms, per_launch=per_launch,
                        achieved=achieved, passes=pst["passes"] / max(1, pst["steps"]),
                        tile_marches=pst["tile_marches"], kernel=kname)

    if rank == 0:
        traffic, tsrc = read_pmc(args.pmc_file, nx, rows)
        out = {
            "metric": "Mcell-updates/s (fp64) for 2D Burgers FOM; % HBM roofline at 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "Mcell-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: reference initial state w0=1, mu=(5.19,0.026), dt=0.05",
            "config": {
                "workload": f"implicit 2D inviscid Burgers FOM, {nx}x{rows} cells per GPU "
                            f"(grid {nx}x{ny}), fp64, exact implicit step (HIP march)",
                "nx": nx, "ny": ny, "rows_per_gpu": rows, "parallelism": f"row-slab x{world}",
                "solver": "march", "engine": args.engine,
            },
            "engine": {"name": args.engine, "stream_w": st["stream_w"],
                       "tiles": st["stream_tiles"], "stall_spins": st["stall_spins"],
                       "slow_diagonals": st["slow_diagonals"],
                       "passes_per_step": st["passes"] / max(1, st["steps"]),
                       "unconverged_steps": st["unconverged_steps"],
                       "device_loop_ms": round(st["loop_ms"], 3)},
        }
        if prof:
            out["roofline"] = {
                "bound": "hbm", "achieved": round(prof["achieved"], 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(prof["achieved"] / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "kernel": prof["kernel"],
                "per_launch_alg_bytes": int(prof["per_launch"]),
                "avg_launch_ms": round(prof["avg_ms"], 5),
                "launches": prof["launches"],
                "traffic_source": tsrc,
            }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(nx, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
