"""Instruction counts of the pipe kernel's diagonal, from its gfx950 ISA.

Compiles finitedifference_amd/csrc/pipe.hip with -save-temps, takes the
unrolled fast-path blocks of pipe_kernel<W, SWEEP> (runs of the code between
consecutive v_rsq_f64 of the cell chain, block overhead included) and counts
instructions by kind, averaged per diagonal.
Writes profiles/<round>/pipe_isa.json, which bench.py turns into the
`issue` roofline: one wave alone issues at most one instruction per 4 cycles
(fp64 FMA measured at 4.3, v_rsq_f64 / v_rcp_f64 at ~16: tools/probes/
issue_probe.hip), so 4 cycles x instructions (+12 per transcendental) is the
per-diagonal floor of a compute wave.

    python tools/isa_count.py [--out profiles/r02/pipe_isa.json]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "finitedifference_amd", "csrc", "pipe.hip")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
         "-Wno-bitwise-instead-of-logical",
         "-mllvm", "-amdgpu-sched-strategy=max-ilp"]  # as the Makefile builds pipe.hip
FLAGS_NARROW = FLAGS  # (round 3: both pipe units use max-ilp, Makefile)
SRC_NARROW = os.path.join(ROOT, "finitedifference_amd", "csrc", "pipe_narrow.hip")


def kind(op):
    if op in ("v_rsq_f64_e32", "v_rcp_f64_e32", "v_sqrt_f64_e32"):
        return "trans_f64"
    if op.startswith("v_") and "_f64" in op:
        return "valu_f64"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_")):
        return "vmem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def kernel_body(asm, W, sweep):
    name = f"_ZN4burg12_GLOBAL__N_111pipe_kernelILi{W}ELb{1 if sweep else 0}EEEvNS_8PipeArgsE:"
    i = asm.index(name)
    return asm[i:asm.index(".Lfunc_end", i)].split("\n")


def runs(lines):
    """Unrolled fast-path blocks: maximal runs of consecutive segments between
    v_rsq_f64 of the cell chain that are not IEEE re-runs (v_div_scale /
    v_div_fixup of the compiler's division).  The last segment of a run also
    holds the loop tail and the next block's head (readiness check, loads);
    the readiness-wait loop (nested loop depth >= 2) is not counted (round 3:
    round 2's counts included it)."""
    rs = [k for k, l in enumerate(lines) if "v_rsq_f64" in l]
    out, cur = [], []
    for a, b in zip(rs, rs[1:] + [len(lines)]):
        seg = lines[a:b]
        if any("v_div_" in l for l in seg):
            if cur:
                out.append(cur)
            cur = []
            continue
        # skip the readiness-wait loop (basic blocks nested at loop depth >= 2:
        # code that runs only while a block waits, not per diagonal)
        ins, inner = [], False
        for l in seg:
            t = l.strip()
            if t.startswith(".LBB"):
                m = re.search(r"Depth=(\d+)", t)
                inner = bool(m) and int(m.group(1)) >= 2
                continue
            if t and not t.startswith((".", ";")) and not inner:
                ins.append(t.split()[0])
        cur.append(ins)
    if cur:
        out.append(cur)
    return [r for r in out if len(r) >= 4]


def summarise(run):
    """Per-block totals of one unrolled run (U diagonals)."""
    c = collections.Counter()
    for ins in run:
        c.update(kind(op) for op in ins)
    n = len(run)
    r = {k: round(v / n, 2) for k, v in sorted(c.items())}
    r["total"] = round(sum(len(i) for i in run) / n, 2)
    r["issue_cycles"] = round(4 * r["total"] + 12 * r.get("trans_f64", 0), 1)
    r["diagonals"] = n
    r["inner_diagonal_total"] = sorted(len(i) for i in run[:-1])[(n - 1) // 2]
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02", "pipe_isa.json"))
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        # pipe.hip (wide kernels) and pipe_narrow.hip (narrow), both with
        # max-ilp, as the Makefile builds them
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "-c", SRC, "-o", os.path.join(d, "p.o"),
                        "-save-temps"], cwd=d, check=True, capture_output=True)
        asm = open(os.path.join(d, "pipe-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS_NARROW, "-c", SRC_NARROW, "-o",
                        os.path.join(d, "n.o"), "-save-temps"], cwd=d, check=True,
                       capture_output=True)
        asm += open(os.path.join(d, "pipe_narrow-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
    res = {"source": "tools/isa_count.py (hipcc -O3 --offload-arch=gfx950 -save-temps of pipe.hip)",
           "issue_model": "4 cycles per instruction + 12 per fp64 transcendental (one wave per SIMD)"}
    for W, sweep in ((256, False), (16, True), (16, False)):
        U = 8  # diagonals per block (pipe.hip: uw_of / BURG_NARROW_U, 8 since round 3)
        rr = [r[i:i + U] for r in runs(kernel_body(asm, W, sweep)) for i in range(0, len(r), U)]
        rr = sorted([r for r in rr if len(r) == U], key=lambda r: sum(map(len, r)))
        # wide tiles: steady / interior / edge block variants, shortest first
        names = {1: ["block"], 2: ["steady_edge_block", "edge_block"] if W <= 16 else
                 ["interior_block", "edge_block"],
                 3: ["steady_block", "interior_block", "edge_block"],
                 4: ["steady_block", "interior_block", "steady_edge_block", "edge_block"]}[len(rr)]
        res[f"pipe_kernel<{W}, {'true' if sweep else 'false'}>"] = {
            "per_diagonal_averages": {nm: summarise(r) for nm, r in zip(names, rr)}}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
