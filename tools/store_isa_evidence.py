"""The ISA evidence of DESIGN.md section 6.2: compile
pipe.hip of a git revision (default 9afe1a7, the last build before the
store-VGPR fix) with the race-screen knob that exposed the failure
(-DBURG_COMM_PRIO=2), and print

  * the failing window: the W = 256 ring store `buffer_store_dwordx4
    v[62:65], ...` whose data registers the next cell's `v_mul_f64 v[62:63],
    v[66:67], 0.5` rewrote (the wrong cells held 0.5 = 0.5 * pu), with every
    instruction between them;
  * for every dwordx4 store of the pipe kernels, the shortest distance (any
    control-flow path, tools/store_reuse_check.py) to a rewrite of its DATA
    and of its ADDRESS VGPRs, split by the store's soffset form (constant 0,
    the class LLVM's hazard recognizer pads with 2 wait states, vs an SGPR);
  * whether the compiler put an s_nop after any such store.

    python tools/store_isa_evidence.py [REV] > profiles/r06/store_hazard/evidence_REV.txt
"""
import collections
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import store_reuse_check as S  # noqa: E402


def compile_rev(rev, d, knobs=("-DBURG_COMM_PRIO=2",)):
    if rev == "worktree":
        src = os.path.join(ROOT)
    else:
        src = os.path.join(d, "src")
        os.makedirs(src)
        tar = subprocess.run(["git", "-C", ROOT, "archive", rev, "finitedifference_amd/csrc", "include"],
                             check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", src], input=tar, check=True)
    csrc = os.path.join(src, "finitedifference_amd", "csrc")
    out = os.path.join(d, "pipe.s")
    flags = [f for f in S.BASE if f not in (S.CSRC, os.path.join(ROOT, "include"))]
    flags = [f for f in flags if f != "-I"]
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, *S.MAXILP, *knobs, "-I", csrc, "-I",
                    os.path.join(src, "include"), os.path.join(csrc, "pipe.hip"), "-o", out],
                   check=True, capture_output=True)
    return open(out).read()


def main():
    rev = sys.argv[1] if len(sys.argv) > 1 else "9afe1a7"
    with tempfile.TemporaryDirectory() as d:
        asm = compile_rev(rev, d)
    ks = S.kernels(asm)
    print(f"# pipe.hip at {rev}, -DBURG_COMM_PRIO=2, gfx950 (hipcc {S.BASE[0]} ... max-ilp)")
    shown = False
    for name, (insts, labels) in ks.items():
        if "pipe_kernelILi256" not in name or shown:
            continue
        for i, ins in enumerate(insts):
            if not (ins.startswith("buffer_store_dwordx4 v[62:65]") and "sc1" in ins):
                continue
            for j in range(i + 1, min(len(insts), i + 20)):
                if insts[j].startswith("v_mul_f64 v[62:63], v[66:67], 0.5"):
                    print(f"\n## the failing window ({name})")
                    for k in range(i, j + 1):
                        print(f"  {k - i:+3d}  {insts[k]}")
                    shown = True
                    break
            if shown:
                break
    print("\n## shortest rewrite after each dwordx4 store of the pipe kernels (any path)")
    print("## distance buckets of 3: count")
    for form in ("soffset 0", "soffset SGPR"):
        for what in ("data", "address"):
            hist = collections.Counter()
            n = 0
            for name, (insts, labels) in ks.items():
                if "pipe_kernel" not in name:
                    continue
                for i, ins in enumerate(insts):
                    op, ops = S.parse(ins)
                    if op != "buffer_store_dwordx4":
                        continue
                    so = ops[3].split()[0] if len(ops) > 3 else ""
                    if (so == "0") != (form == "soffset 0"):
                        continue
                    n += 1
                    regs = S.vregs(ops[0]) if what == "data" else S.vregs(ops[1])
                    hit = S.scan(insts, labels, i, regs, 200) if regs else None
                    hist["none" if hit is None else min(hit[0], 60) // 3 * 3] += 1
            items = sorted(((k, v) for k, v in hist.items() if k != "none"))
            print(f"{form:13s} {what:8s} stores {n:5d}: " +
                  " ".join(f"{k}-{k + 2}:{v}" for k, v in items[:10]) +
                  (f" ... none<=200:{hist['none']}" if hist["none"] else ""))
    nops = sum(1 for _, (insts, _) in ks.items() for i, x in enumerate(insts[:-1])
               if x.startswith("buffer_store_dwordx4") and insts[i + 1].startswith("s_nop"))
    print(f"\ndwordx4 stores followed by an s_nop: {nops}")


if __name__ == "__main__":
    main()
