#!/bin/bash
# A/B: north hand-offs to same-GPU mailboxes with agent-scope stores
# (libburgers_hip_nag.so, -DBURG_NORTH_AGENT=1) vs the default system-scope
# flavour: the mailbox / halo tests on the variant, then the 4096^2 headline
# (3 steps), the 1024^2 9-mu sweep and one 1024^2 trajectory, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab_nag}; mkdir -p $O
BURG_LIB=$PWD/finitedifference_amd/libburgers_hip_nag.so timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "pair or sweep_each or pipe_1024 or pipe_bitwise_sequential or slab_halo or wide" > $O/pytest_nag.log 2>&1 || { tail -30 $O/pytest_nag.log; exit 1; }
tail -1 $O/pytest_nag.log
B4="bench.py --steps 3 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check"
for r in 1 2 3; do for v in base nag; do
  L=$PWD/finitedifference_amd/libburgers_hip.so; [ $v = nag ] && L=$PWD/finitedifference_amd/libburgers_hip_nag.so
  BURG_LIB=$L timeout -k 10 300 python3 $B4 2>> $O/ab.err | python3 -c "
import sys, json
b = json.loads(sys.stdin.read().strip().splitlines()[-1])
print(json.dumps({'v': '$v', 'r': $r, 'headline': b['value'], 'kernel_ms': b['roofline']['avg_launch_ms']}))" >> $O/ab.jsonl || { tail -5 $O/ab.err; exit 1; }
  BURG_LIB=$L timeout -k 10 300 python3 -c "
import json, bench
c = bench.config2_1024(None)
s = bench.single_1024(None, None)
print(json.dumps({'v': '$v', 'r': $r, 'sweep_ms': c['avg_launch_ms'], 'single_ms': s['avg_launch_ms']}))
" >> $O/ab.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done; done
cat $O/ab.jsonl
echo ABOK
