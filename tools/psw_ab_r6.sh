#!/bin/bash
# The paired kernel's store wave: the whole GPU
# suite on the default build, then the 1024^2 9-mu sweep (bench.config2_1024)
# and one 1024^2 x 500 trajectory, default build vs the previous one
# (libburgers_hip_prev.so, built from the sources before the change),
# 3 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab_psw}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do for v in prev new; do
  L=$PWD/finitedifference_amd/libburgers_hip.so; [ $v = prev ] && L=$PWD/finitedifference_amd/libburgers_hip_prev.so
  BURG_LIB=$L timeout -k 10 300 python3 -c "
import json, bench
c = bench.config2_1024(None)
print(json.dumps({'v': '$v', 'r': $r, 'sweep_ms': c['avg_launch_ms'], 'sweep_value': c['value'], 'paired': c['paired_halves'], 'ieee': c['ieee_diagonals']}))
" >> $O/ab.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done; done
cat $O/ab.jsonl
echo ABOK
