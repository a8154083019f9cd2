"""Roofline probe of the HBM-bound stencils (residual K1, J.x K2) alone:
prints bench.py's stencil_roofline object for an nx x nx grid.  Used under
rocprofv3 (--kernel-trace --stats, and the FETCH_SIZE / WRITE_SIZE passes)
so the committed profiles/ summaries come from exactly these launches.

    python tools/stencil_probe.py [nx] [reps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

nx = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
print(json.dumps(bench.stencil_roofline(nx, reps)), flush=True)
