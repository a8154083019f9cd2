"""Instruction counts of the pipe kernel's diagonal, from its gfx950 ISA.

Compiles finitedifference_amd/csrc/pipe.hip and pipe_narrow.hip with
-save-temps (as the Makefile builds them), splits each pipe_kernel<W, SWEEP>
into basic blocks and, for every fast block of U diagonals (U consecutive
v_rsq_f64 of the cell chain outside the IEEE re-run and the readiness-wait
loop), counts the instructions of one loop iteration through it: the
cheapest path over hot blocks from the compute loop's header to the block's
first diagonal, diagonal to diagonal, and back (round 3; until then the code
between consecutive v_rsq_f64 in layout order, which also counted cold code
the compiler placed there).  The cheapest path may skip guarded blocks a wave
does run, so the counts are lower bounds.  Averaged per diagonal by kind.
Writes profiles/<round>/pipe_isa.json, which bench.py turns into the
`issue` roofline: one wave alone issues at most one instruction per 4 cycles
(fp64 FMA measured at 4.3, v_rsq_f64 / v_rcp_f64 at ~16: tools/probes/
issue_probe.hip), so 4 cycles x instructions (+12 per transcendental) is the
per-diagonal floor of a compute wave.

    python tools/isa_count.py [--out profiles/r03/pipe_isa.json]
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


def kernel_body(asm, W, sweep, pair=False):
    # (round 5: pipe_kernel<W, SWEEP, PAIR>)
    name = (f"_ZN4burg12_GLOBAL__N_111pipe_kernelILi{W}ELb{1 if sweep else 0}"
            f"ELb{1 if pair else 0}EEEvNS_8PipeArgsE:")
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


def parse_blocks(lines):
    """Basic blocks of a kernel body: label -> block, in layout order.  Each
    block: its instructions (opcode strings), loop depth, whether it is cold
    (the IEEE re-run, the readiness-wait loop, abort paths), successors."""
    blocks, cur = [], None

    def start(label, depth):
        b = {"label": label, "ins": [], "depth": depth, "succ": []}
        blocks.append(b)
        return b

    for ln in lines:
        t = ln.strip()
        is_lbl = t.startswith(".LBB") and t.split()[0].endswith(":")
        if is_lbl or t.startswith("; %bb."):
            m = re.search(r"Depth=(\d+)", t)
            label = t.split()[0].rstrip(":") if is_lbl else None
            cur = start(label, int(m.group(1)) if m else 0)
            if re.search(r"Loop Header: Depth=1\b", t):
                cur["header"] = True
            continue
        if not t or t.startswith((".", ";")):
            if cur is not None and re.search(r"Loop Header: Depth=1\b", t):
                cur["header"] = True  # (the header comment on its own line)
            continue
        if cur is None or (cur["ins"] and cur["ins"][-1].startswith(("s_branch", "s_cbranch"))):
            cur = start(None, cur["depth"] if cur else 0)
        cur["ins"].append(t.split()[0] if not t.startswith(("s_branch", "s_cbranch")) else t)
    idx = {b["label"]: i for i, b in enumerate(blocks) if b["label"]}
    for i, b in enumerate(blocks):
        last = b["ins"][-1] if b["ins"] else ""
        nxt = [i + 1] if i + 1 < len(blocks) else []
        if last.startswith("s_branch"):
            b["succ"] = [idx[last.split()[1]]]
        elif last.startswith("s_cbranch"):
            b["succ"] = [idx[last.split()[1]]] + nxt
        elif last.startswith(("s_endpgm", "s_setpc")):
            b["succ"] = []
        else:
            b["succ"] = nxt
        b["ins"] = [x.split()[0] for x in b["ins"]]
        b["cold"] = b["depth"] >= 2 or any(
            o.startswith(("v_div_scale", "v_div_fixup"))
            for o in b["ins"])
    return blocks


def hot_cycle(blocks, U):
    """Per fast run of U diagonals (U consecutive v_rsq_f64 outside the cold
    blocks): the instructions one loop iteration through that run executes --
    the cheapest path over hot blocks from the compute loop's header to the
    run's first diagonal, from diagonal to diagonal, and back to the header
    (routing never passes the header in between).  Returns per-diagonal
    opcode lists (the header-to-first-rsq and last-rsq-to-header code in the
    last diagonal's list, as runs() does)."""
    import heapq
    rsq = [(i, j) for i, b in enumerate(blocks) if not b["cold"]
           for j, o in enumerate(b["ins"]) if o.startswith("v_rsq_f64")]
    # the compute loop's header: of the depth-1 loop headers, the one the
    # most runs close a cycle through (the comm and loader loops close none)
    best = []
    for H in [i for i, b in enumerate(blocks) if b.get("header")]:
        r = _cycles(blocks, U, rsq, H)
        if len(r) > len(best):
            best = r
    return best


def _cycles(blocks, U, rsq, H):
    import heapq

    def path(a, z):
        # the CHEAPEST a -> z path over hot blocks (z's instructions included,
        # a's not; never through the header in between): a lower bound of
        # what a wave executes -- guarded blocks a wave does run (an
        # exec-masked store, a check of an edge it has) may be skipped, so the
        # issue roofline built on this count is conservative
        dist, prev, pq = {a: 0}, {}, [(0, a)]
        while pq:
            d, u = heapq.heappop(pq)
            if u == z and u in prev:
                break
            if d > dist.get(u, 1 << 60):
                continue
            for v in blocks[u]["succ"]:
                if blocks[v]["cold"] or (v == H and z != H):
                    continue
                nd = d + len(blocks[v]["ins"]) + 1
                if nd < dist.get(v, 1 << 60) or (v == z and v == a and v not in prev):
                    dist[v], prev[v] = nd, u
                    heapq.heappush(pq, (nd, v))
        if z not in prev:
            return None
        out, v = [z], prev[z]
        while v != a:
            out.append(v)
            v = prev[v]
        return out[::-1]

    # group the hot rsq's into runs of U (in layout order)
    res = []
    for g in range(0, len(rsq) - U + 1, U):
        run = rsq[g:g + U]
        seq = [H] + (path(H, run[0][0]) or [])
        ok = len(seq) > 1 or run[0][0] == H
        for (b0, _), (b1, _) in zip(run, run[1:]):
            p = path(b0, b1) if b1 != b0 else []
            if p is None:
                ok = False
                break
            seq += p
        back = path(run[-1][0], H)
        if not ok or back is None:
            continue
        seq += back[:-1]  # (the header is seq[0])
        ops = [o for bi in seq for o in blocks[bi]["ins"]]
        # rotate to start at the run's first rsq, split at each rsq
        pos = [k for k, o in enumerate(ops) if o.startswith("v_rsq_f64")]
        if len(pos) != U:
            continue
        ops = ops[pos[0]:] + ops[:pos[0]]
        pos = [p - pos[0] for p in pos] + [len(ops)]
        res.append([ops[pos[i]:pos[i + 1]] for i in range(U)])
    return res


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
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06", "pipe_isa.json"))
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
    for W, sweep, pair in ((256, False, False), (16, True, False), (16, False, False),
                           (16, False, True), (16, True, True)):
        # diagonals per block (pipe.hip: uw_of / BURG_NARROW_U): 16 for wide
        # tiles of 128 and 256 columns, 8 otherwise (round 3); the paired
        # kernel (round 5) runs two cell chains per diagonal: its 8-diagonal
        # block holds 16 v_rsq_f64, counted here per CELL (x 2 per diagonal)
        U = 16 if W in (128, 256) or pair else 8
        rr = hot_cycle(parse_blocks(kernel_body(asm, W, sweep, pair)), U)
        rr = sorted([r for r in rr if len(r) == U], key=lambda r: sum(map(len, r)))
        # wide tiles: steady / interior / edge block variants, shortest first
        # (steady-edge blocks are built twice since round 3: for the
        # workgroup's east wave -- "_east", outflow to the global mailbox --
        # and for the others; the two differ by a store and a select)
        names = {1: ["block"], 2: ["steady_edge_block", "edge_block"] if W <= 16 else
                 ["interior_block", "edge_block"],
                 3: ["steady_edge_block", "steady_edge_block_east", "edge_block"] if W <= 16 else
                 ["steady_block", "interior_block", "edge_block"],
                 4: ["steady_block", "interior_block", "steady_edge_block", "edge_block"],
                 5: ["steady_block", "interior_block", "steady_edge_block", "steady_edge_block_east",
                     "edge_block"]}[len(rr)]
        res[f"pipe_kernel<{W}, {'true' if sweep else 'false'}{', paired (per cell)' if pair else ''}>"] = {
            "per_diagonal_averages": {nm: summarise(r) for nm, r in zip(names, rr)}}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
