"""Store-VGPR hazard check: compile the pipe kernels
to gfx950 assembly (as the Makefile builds them) and require that no
buffer_store's data or offset VGPRs are rewritten within MIN straight-line
instructions after the store (round 5: a store that read its VGPRs late,
under memory-pipeline load, stored the next cell's value).

    python tools/store_reuse_check.py [MIN]   -> exit 1 and the sites if any
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "finitedifference_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
         "-Wno-bitwise-instead-of-logical", "-mllvm", "-amdgpu-sched-strategy=max-ilp",
         "--cuda-device-only", "-S", "-I", CSRC, "-I", os.path.join(ROOT, "include")]


def written(ins):
    parts = ins.split(None, 1)
    if len(parts) < 2:
        return set()
    op, rest = parts
    if op.startswith(("s_", "buffer_store", "ds_write", "global_store", "buffer_atomic", "global_atomic")):
        return set()
    if op.startswith("v_cmp") and op.endswith("e32"):
        return set()
    dst = rest.split(",")[0].strip()
    m = re.match(r"v\[(\d+):(\d+)\]", dst)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", dst)
    return {int(m.group(1))} if m else set()


def check(asm, min_dist):
    bad = []
    for m in re.finditer(r"^(_ZN4burg12_GLOBAL__N_111pipe_kernel\w+):", asm, re.M):
        body = asm[m.end():asm.index(".Lfunc_end", m.end())]
        L = [l.strip() for l in body.split("\n")
             if l.strip() and not l.strip().startswith((".", ";")) and not l.strip().endswith(":")]
        for a, ins in enumerate(L):
            s = re.match(r"buffer_store_dwordx4 v\[(\d+):(\d+)\], v(\d+)", ins)
            if not s:
                continue
            regs = set(range(int(s.group(1)), int(s.group(2)) + 1)) | {int(s.group(3))}
            for b in range(a + 1, min(len(L), a + min_dist)):
                if L[b].startswith(("s_branch", "s_cbranch", "s_endpgm")):
                    break
                if written(L[b]) & regs:
                    bad.append((m.group(1), b - a, ins, L[b]))
                    break
    return bad


def main():
    min_dist = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    bad = []
    with tempfile.TemporaryDirectory() as d:
        for src in ("pipe.hip", "pipe_narrow.hip"):
            out = os.path.join(d, src + ".s")
            subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, os.path.join(CSRC, src), "-o", out], check=True,
                           capture_output=True)
            bad += check(open(out).read(), min_dist)
    for k, dist, st, w in bad:
        print(f"{k}: {st}  rewritten {dist} later by  {w}")
    print(f"store VGPR reuse within {min_dist} instructions: {len(bad)} sites")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
