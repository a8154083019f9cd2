#!/bin/bash
# The paired store wave's two ring layouts: the
# 1024^2 9-mu sweep with the paired sweep layout (default), with the standard
# layout (BURG_PAIR_LAYOUT=0), and the previous build, 3 rounds, with the
# compute waves' wait statistics.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab_play}; mkdir -p $O
for r in 1 2 3; do for v in prev lay std; do
  L=$PWD/finitedifference_amd/libburgers_hip.so; [ $v = prev ] && L=$PWD/finitedifference_amd/libburgers_hip_prev.so
  PL=1; [ $v = std ] && PL=0
  BURG_PAIR_LAYOUT=$PL BURG_LIB=$L timeout -k 10 300 python3 -c "
import json, bench, numpy as np
from finitedifference_amd.config import get_snapshot_params
from finitedifference_amd.solver import FOMContext
nx, T = 1024, 500
mus = get_snapshot_params()[:9]
ctx = FOMContext(nx, nx, engine='pipe')
g = np.linspace(0, 100, nx + 1)
ctx.set_problem(g, g, bench.DT, bench.MU)
ctx.upload(np.ones(ctx.m))
ctx.sweep(mus, T, keep_snaps=False)
ms = []
for _ in range(3):
    st = ctx.sweep(mus, T, keep_snaps=False)[1]
    ms.append(st['loop_ms'])
ctx.close()
keys = ('stall_spins', 'slow_diagonals', 'slow_ticks', 'ramp_ms', 'paired_launches')
print(json.dumps({'v': '$v', 'r': $r, 'sweep_ms': round(sum(ms) / 3, 4), **{k: st[k] for k in keys}}))
" >> $O/ab.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done; done
cat $O/ab.jsonl
echo ABOK
