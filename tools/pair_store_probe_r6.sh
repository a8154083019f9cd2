#!/bin/bash
# Ceiling / layout probes of the paired sweep kernel's ring stores (DESIGN.md
# section 4.1f'): the 1024^2 9-mu sweep (bench.config2_1024) on the default
# build and on each named variant (libburgers_hip_NAME.so; wrong ring
# contents: -DBURG_AB_PAIR_NORING=1 "pnr", -DBURG_AB_PAIR_COAL=1 "pcoal",
# -DBURG_AB_PAIR_OOB=1 "poob", -DBURG_AB_PAIR_NOKEEP=1 "pnk"; cache policy
# -DBURG_RING_ST_AUX=2 "pnt"), 3 interleaved rounds, with the launch's wait
# statistics.
#   TAG=ab_x tools/pair_store_probe_r6.sh pnr pcoal
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab_pstore}; mkdir -p $O
for r in 1 2 3; do for v in base "$@"; do
  L=$PWD/finitedifference_amd/libburgers_hip.so; [ $v != base ] && L=$PWD/finitedifference_amd/libburgers_hip_$v.so
  BURG_LIB=$L timeout -k 10 300 python3 -c "
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
keys = ('stall_spins', 'slow_diagonals', 'slow_ticks', 'comm_polls', 'ramp_ms', 'ieee_diagonals', 'paired_launches')
print(json.dumps({'v': '$v', 'r': $r, 'sweep_ms': round(sum(ms) / 3, 4), **{k: st[k] for k in keys}}))
" >> $O/ab.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done; done
cat $O/ab.jsonl
echo ABOK
