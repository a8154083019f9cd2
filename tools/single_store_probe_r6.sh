#!/bin/bash
# Ceiling probe of the ring stores for one 1024^2 x 500 trajectory (the
# one-cell W = 16 kernel with its store wave): default build vs the store
# wave without stores (libburgers_hip_swns.so, -DBURG_AB_SW_NOSTORE=1, wrong
# ring contents), 3 interleaved rounds (bench.single_1024).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab_swns}; mkdir -p $O
for r in 1 2 3; do for v in base swns; do
  L=$PWD/finitedifference_amd/libburgers_hip.so; [ $v != base ] && L=$PWD/finitedifference_amd/libburgers_hip_$v.so
  BURG_LIB=$L timeout -k 10 300 python3 -c "
import json, bench
s = bench.single_1024(None, None)
print(json.dumps({'v': '$v', 'r': $r, 'single_ms': s['avg_launch_ms'], 'ramp_ms': s['ramp_ms']}))
" >> $O/ab.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done; done
cat $O/ab.jsonl
echo ABOK
