#!/bin/bash
# The one-cell store wave in the paired store wave's form (scalar entry
# offsets for full blocks, vmcnt drains instead of kept copies; DESIGN.md
# section 4.1g): the whole GPU suite, then one 1024^2 x 500 trajectory
# (bench.single_1024) and the one-cell 9-mu sweep (BURG_PAIR=0), default
# build vs the previous one (libburgers_hip_prev.so), 3 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab_swc}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do for v in prev new; do
  L=$PWD/finitedifference_amd/libburgers_hip.so; [ $v = prev ] && L=$PWD/finitedifference_amd/libburgers_hip_prev.so
  BURG_LIB=$L timeout -k 10 300 python3 -c "
import json, bench
s = bench.single_1024(None, None)
print(json.dumps({'v': '$v', 'r': $r, 'single_ms': s['avg_launch_ms'], 'ramp_ms': s['ramp_ms']}))
" >> $O/ab.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
  BURG_PAIR=0 BURG_LIB=$L timeout -k 10 300 python3 -c "
import json, bench
c = bench.config2_1024(None)
print(json.dumps({'v': '$v', 'r': $r, 'sweep_onecell_ms': c['avg_launch_ms']}))
" >> $O/ab.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done; done
cat $O/ab.jsonl
echo ABOK
