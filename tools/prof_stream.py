"""One 1024^2 streaming advance for PMC profiling (diagnostics)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from finitedifference_amd.solver import FOMContext
nx = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
K = int(sys.argv[2]) if len(sys.argv) > 2 else 550
c = FOMContext(nx, nx, stream_w=int(os.environ.get("W", "16")))
c.set_problem(np.linspace(0, 100, nx + 1), np.linspace(0, 100, nx + 1), 0.05, (5.19, 0.026))
c.upload(np.ones(2 * nx * nx))
st = c.advance(K)
print("loop_ms", st["loop_ms"], "spins", st["stall_spins"])
