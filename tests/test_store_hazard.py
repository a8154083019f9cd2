"""CPU: the pipe kernels' gfx950 assembly keeps every buffer store's data
and offset VGPRs unwritten for 40 straight-line instructions after the store
(a store that read its VGPRs late, under memory-
pipeline load, stored the next cell's value -- wrong ring entries).
Compiles pipe.hip and pipe_narrow.hip with hipcc (no GPU needed)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_store_vgpr_reuse_in_pipe_kernels():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "store_reuse_check.py"), "40"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 sites" in r.stdout


def test_narrow_w8_run_kernel_fits_four_waves_per_simd():
    """The W = 8 run kernel puts three 5-wave workgroups on a CU (the 750^2
    eight-slab case on one GPU): its VGPRs must allow 4 waves per SIMD
    (<= 128; round 5's store-VGPR fix had raised it to 132 and that GPU
    test then timed out), with no scratch."""
    import re
    src = os.path.join(ROOT, "finitedifference_amd", "csrc", "pipe_narrow.hip")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                        "-ffp-contract=off", "-Wno-bitwise-instead-of-logical", "-mllvm",
                        "-amdgpu-sched-strategy=max-ilp", "--cuda-device-only", "-c", src, "-o", os.devnull,
                        "-I", os.path.join(ROOT, "finitedifference_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    names = re.findall(r"Function Name: (\S+)", r.stderr)
    vgprs = [int(x) for x in re.findall(r"\bVGPRs: (\d+)", r.stderr)]
    scratch = [int(x) for x in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", r.stderr)]
    found = False
    for n, v, sc in zip(names, vgprs, scratch):
        if "pipe_kernelILi8ELb0E" in n:
            found = True
            assert v <= 128 and sc == 0, (n, v, sc)
    assert found
