#!/bin/bash
# GPU pass for the ECSW kernel: parity tests, probe, rocprofv3 stats of the probe.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-ecsw}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 200 python tools/ecsw_probe.py 250 95 50 > $O/ecsw_probe.json 2> $O/ecsw_probe.err || { tail -20 $O/ecsw_probe.err; exit 1; }
cat $O/ecsw_probe.json
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ecsw -o run -- python3 $R/tools/ecsw_probe.py 250 95 20 > $O/prof_ecsw.log 2>&1 || { tail -20 $O/prof_ecsw.log; exit 1; }
tail -1 $O/prof_ecsw.log
echo ALLOK
