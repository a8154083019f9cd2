#!/bin/bash
# Where the paired kernel (with its store wave) starts to beat the one-cell
# kernel for ONE trajectory (pipe_args' threshold K >= (nx + rows) / 2):
# 1024^2 x 300 / 500 / 800 steps, BURG_PAIR=0 vs 1, 3 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pthr}; mkdir -p $O
for r in 1 2 3; do for T in 300 500 800; do for P in 0 1; do
  BURG_PAIR=$P timeout -k 10 300 python3 -c "
import json, bench, numpy as np
from finitedifference_amd.solver import FOMContext
nx, T = 1024, $T
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
print(json.dumps({'T': T, 'pair': $P, 'r': $r, 'ms': round(sum(ms) / 3, 4), 'paired': st['paired_launches']}))
" >> $O/ab.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done; done; done
cat $O/ab.jsonl
echo ABOK
