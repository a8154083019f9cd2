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
