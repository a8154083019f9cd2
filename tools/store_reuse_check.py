"""Store-VGPR reuse check: compile the product
kernels to gfx950 assembly (as the Makefile builds them) and require that no
vector-memory store's data or address VGPRs are rewritten within MIN
instructions after the store, along EVERY control-flow path -- through
fall-through, taken branches and loop back-edges (round 5: a ring store whose
data registers were rewritten 9 instructions later stored the next cell's
value under memory-pipeline load; the compiler's hazard window for a
dwordx3/x4 store is 2 wait states).

What counts:
  * stores: every buffer_store*, global_store*, flat_store*, scratch_store*
    and buffer/global atomic with data wider than 64 bits -- the class LLVM's
    gfx9 hazard recognizer pads (GCNHazardRecognizer::createsVALUHazard: 2
    wait states on gfx940+) and the class that failed (dwordx4) -- their data
    VGPRs and their VGPR address or offset when they have one (`off` / an
    SGPR-only offset has none); narrower stores are counted in --report;
  * a rewrite: any instruction whose destination is one of those VGPRs
    (VALU, VMEM / LDS loads; LDS-DMA loads and stores write none);
  * a path ends safely at an `s_waitcnt vmcnt(0)` (the store has completed)
    or at s_endpgm;
  * distance: instructions after the store along the path (labels and
    directives do not count).

    python tools/store_reuse_check.py [MIN] [--all] [--report]
      MIN       the threshold (default 24: DESIGN.md section 6.2 -- the failing
                round-5 build had 9, the screened builds >= 29)
      --all     also fail on the kernels that are not screened (default: only
                the march kernels -- pipe, stream -- must pass; the others are
                reported)
      --report  print every kernel's store count and shortest distance
Exit 1 when a checked kernel has a store below MIN (its sites are printed).
"""
import os
import re
import subprocess
import sys
import tempfile
from collections import deque

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "finitedifference_amd", "csrc")
BASE = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
        "-Wno-bitwise-instead-of-logical", "--cuda-device-only", "-S", "-I", CSRC,
        "-I", os.path.join(ROOT, "include")]
MAXILP = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
# (source, extra flags as the Makefile builds it, must-pass kernel name pattern)
UNITS = [("pipe.hip", MAXILP, r"pipe_kernel"),
         ("pipe_narrow.hip", MAXILP, r"pipe_kernel"),
         ("stream.hip", [], r"stream_kernel"),
         ("stencil.hip", [], None), ("march.hip", [], None), ("ecsw.hip", [], None),
         ("lspg.hip", [], None), ("pod.hip", [], None)]

STORE = re.compile(r"^(buffer|global|flat|scratch)_(store|atomic)\w*$")


def split_ops(rest):
    """Operands of an instruction (commas inside [] do not split)."""
    out, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def vregs(tok):
    tok = tok.split()[0] if tok else ""
    m = re.match(r"v\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def parse(ins):
    parts = ins.split(None, 1)
    return parts[0], (split_ops(parts[1]) if len(parts) > 1 else [])


def store_regs(op, ops):
    """(VGPRs a store reads after issue: data + VGPR address / offset,
    data width in dwords)."""
    if op.startswith("buffer_"):
        data, addr = ops[0], (ops[1] if len(ops) > 1 else "")
    else:  # global / flat / scratch: vaddr first, then data
        addr, data = ops[0], (ops[1] if len(ops) > 1 else "")
    return vregs(data) | vregs(addr), len(vregs(data))


def written(op, ops, ins):
    """VGPRs an instruction writes."""
    # (v_cmp* write VCC / an SGPR pair / EXEC; LDS-DMA loads write LDS)
    if not ops or op.startswith(("s_", "ds_write", "ds_store", "v_cmp")) or STORE.match(op) or \
            re.search(r"\slds\b", ins):
        return set()
    w = vregs(ops[0])
    if op.startswith("v_swap"):
        w |= vregs(ops[1]) if len(ops) > 1 else set()
    return w


def kernels(asm):
    """{symbol: (instructions, label -> index)} of every kernel in the file."""
    out = {}
    for m in re.finditer(r"^(_Z\w+):\s*(?:;.*)?$", asm, re.M):
        end = asm.find(".Lfunc_end", m.end())
        if end < 0:
            continue
        body = asm[m.end():end]
        insts, labels = [], {}
        for raw in body.split("\n"):
            line = raw.split(";")[0].strip()
            if not line or line.startswith("."):
                if line.startswith(".LBB") and line.endswith(":"):
                    labels[line[:-1]] = len(insts)
                continue
            if line.endswith(":"):
                labels[line[:-1]] = len(insts)
                continue
            insts.append(line)
        out[m.group(1)] = (insts, labels)
    return out


def successors(i, insts, labels):
    op, ops = parse(insts[i])
    if op == "s_endpgm" or op.startswith("s_setpc") or op.startswith("s_trap"):
        return []
    if op == "s_branch":
        return [labels[ops[0]]] if ops and ops[0] in labels else []
    if op.startswith("s_cbranch"):
        nxt = [i + 1] if i + 1 < len(insts) else []
        return nxt + ([labels[ops[0]]] if ops and ops[0] in labels else [])
    return [i + 1] if i + 1 < len(insts) else []


def drained(ins):
    return ins.startswith("s_waitcnt") and re.search(r"vmcnt\(0\)", ins) is not None


def scan(insts, labels, i, regs, horizon):
    """Shortest path distance (instructions after store i) to a rewrite of
    `regs`, over every control-flow path, or None within `horizon`."""
    best = {}
    q = deque((s, 1) for s in successors(i, insts, labels))
    hit = None
    while q:
        j, d = q.popleft()
        if d > horizon or (j in best and best[j] <= d):
            continue
        best[j] = d
        op, ops = parse(insts[j])
        if written(op, ops, insts[j]) & regs:
            if hit is None or d < hit[0]:
                hit = (d, j)
            continue
        if drained(insts[j]):
            continue
        for s in successors(j, insts, labels):
            q.append((s, d + 1))
    return hit


def check_asm(asm, min_dist, must=None, horizon=None, wide_only=True):
    """[(kernel, stores, shortest, sites, checked)] over the stores of the
    hazard class (wide_only: data wider than 64 bits -- the stores LLVM's
    gfx9 hazard recognizer pads, GCNHazardRecognizer::createsVALUHazard; all
    stores otherwise): sites below min_dist."""
    horizon = horizon or max(min_dist, 64)
    rows = []
    for name, (insts, labels) in kernels(asm).items():
        stores, shortest, sites = 0, None, []
        for i, ins in enumerate(insts):
            op, ops = parse(ins)
            if not STORE.match(op):
                continue
            regs, width = store_regs(op, ops)
            if wide_only and width <= 2:
                continue
            stores += 1
            hit = scan(insts, labels, i, regs, horizon)
            if hit is None:
                continue
            d, j = hit
            shortest = d if shortest is None else min(shortest, d)
            if d < min_dist:
                sites.append((d, ins, insts[j]))
        checked = must is None or re.search(must, name) is not None
        rows.append((name, stores, shortest, sites, checked))
    return rows


def compile_unit(src, extra, d, defines=()):
    out = os.path.join(d, src + ".s")
    subprocess.run(["/opt/rocm/bin/hipcc", *BASE, *extra, *defines, os.path.join(CSRC, src), "-o", out],
                   check=True, capture_output=True)
    return open(out).read()


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    min_dist = int(args[0]) if args else 24
    strict_all = "--all" in sys.argv
    report = "--report" in sys.argv
    bad, total_stores, checked_stores = [], 0, 0
    with tempfile.TemporaryDirectory() as d:
        for src, extra, must in UNITS:
            rows = check_asm(compile_unit(src, extra, d), min_dist,
                             must=None if strict_all else (must or r"^$"))
            for name, stores, shortest, sites, checked in rows:
                total_stores += stores
                if checked:
                    checked_stores += stores
                if report or (checked and sites):
                    print(f"{src}: {name}: {stores} stores, shortest rewrite "
                          f"{'>= horizon' if shortest is None else shortest}"
                          f"{'' if checked else '  (reported only)'}")
                if checked:
                    for dist, st, w in sites:
                        bad.append(name)
                        print(f"    {st}  rewritten {dist} later by  {w}")
    print(f"store VGPR reuse within {min_dist} instructions on any path: {len(bad)} sites "
          f"({checked_stores} stores in the checked kernels, {total_stores} in all)")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
