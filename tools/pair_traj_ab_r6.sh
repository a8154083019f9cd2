#!/bin/bash
# Paired single trajectories after the paired store wave (standard layout,
# per-lane walk, drained per block): the whole GPU
# suite, then one 1024^2 x 1500 trajectory (paired by default: K >= (nx +
# rows) / 2; BURG_PAIR=1 set explicitly) on the default build, on the build before the paired store wave
# (libburgers_hip_prev.so) and one-cell (BURG_PAIR=0), 3 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab_ptraj}; mkdir -p $O
if [ -z "$SKIP_SUITE" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
fi
for r in 1 2 3; do for v in prev new onecell; do
  L=$PWD/finitedifference_amd/libburgers_hip.so; [ $v = prev ] && L=$PWD/finitedifference_amd/libburgers_hip_prev.so
  P=1; [ $v = onecell ] && P=0
  BURG_PAIR=$P BURG_LIB=$L timeout -k 10 300 python3 -c "
import json, bench, numpy as np
from finitedifference_amd.solver import FOMContext
nx, T = 1024, 1500
ctx = FOMContext(nx, nx, engine='pipe')
g = np.linspace(0, 100, nx + 1)
ctx.set_problem(g, g, bench.DT, bench.MU)
ctx.upload(np.ones(ctx.m))
ctx.reserve(T)
ctx.trajectory(T)
ms = []
for _ in range(3):
    st = ctx.trajectory(T)
    ms.append(st['loop_ms'])
ctx.close()
print(json.dumps({'v': '$v', 'r': $r, 'traj1500_ms': round(sum(ms) / 3, 4), 'paired': st['paired_launches'], 'slow': st['slow_diagonals']}))
" >> $O/ab.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done; done
cat $O/ab.jsonl
echo ABOK
