#!/bin/bash
# The whole GPU suite on the final build, then where the 1024^2 kernels'
# compute waves wait (BURG_STREAM_DEBUG=8: blocks that waited by missing
# kind, incl. the store wave): the 9-mu sweep (paired) and one trajectory.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-swdiag}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
BURG_STREAM_DEBUG=8 timeout -k 10 300 python3 -c "
import json, bench
c = bench.config2_1024(None, steps=1)
s = bench.single_1024(None, None, steps=1)
print(json.dumps({'sweep_ms': c['avg_launch_ms'], 'single_ms': s['avg_launch_ms']}))
" > $O/diag.json 2> $O/diag.err || { tail -5 $O/diag.err; exit 1; }
grep "\[pipe\]" $O/diag.err | tail -8
cat $O/diag.json
echo DIAGOK
