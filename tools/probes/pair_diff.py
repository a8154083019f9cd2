"""Where the paired kernel differs from the oracle: python pair_diff.py nx ny T
(BURG_PAIR from the environment); prints the first mismatching cells."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle  # noqa: E402
from test_gpu_regime import _ctx, _problem, planted_w0  # noqa: E402

nx, ny, T = (int(x) for x in sys.argv[1:4])
P = _problem(oracle, nx, ny)
w0 = planted_w0(nx, ny) if os.environ.get("PLANT", "1") == "1" else np.ones(2 * nx * ny)
ref, _, _ = P.fom(w0, T)
ctx = _ctx(nx, ny, engine="pipe", stream_w=16)
snaps, st, _, _ = ctx.run(w0, T)
n = nx * ny
for j in range(1, T + 1):
    bad = np.nonzero(snaps[:, j] != ref[j])[0]
    if len(bad):
        cells = sorted(set(int(b % n) for b in bad))
        rc = [(c // nx, c % nx) for c in cells[:12]]
        print(f"BURG_PAIR={os.environ.get('BURG_PAIR')} step {j}: {len(cells)} cells differ, first (row, col): {rc}")
        rows = sorted(set(c // nx for c in cells)); cols = sorted(set(c % nx for c in cells))
        print(f"  rows {rows[:10]}..{rows[-3:]} ({len(rows)}), cols {cols[:16]}..{cols[-3:]} ({len(cols)})")
        break
else:
    print(f"BURG_PAIR={os.environ.get('BURG_PAIR')}: all {T} steps equal")
# which step's value does a wrong cell hold?
for j in range(1, T + 1):
    bad = np.nonzero(snaps[:, j] != ref[j])[0]
    if len(bad):
        for b in bad[:6]:
            v = snaps[b, j]
            hits = [q for q in range(T + 1) if ref[q][b] == v]
            print(f"  step {j} elem {b} (row {(b % n) // nx}, col {(b % n) % nx}, {'v' if b >= n else 'u'}): "
                  f"gpu {v!r} ref {ref[j][b]!r}; equals ref steps {hits}")
        break
