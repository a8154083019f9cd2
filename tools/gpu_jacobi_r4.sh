#!/bin/bash
# POD with the interleaved Jacobi pairs: tests, probe (and kernel stats)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r4z2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "pod" > $O/pytest_pod.log 2>&1 || { tail -40 $O/pytest_pod.log; exit 1; }
tail -2 $O/pytest_pod.log
POD_PROBE_RSVD_ONLY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pod_stats -o run -- python3 tools/pod_probe.py > $O/pod_probe_prof.json 2> $O/pod_stats.err || { tail -5 $O/pod_stats.err; exit 1; }
POD_PROBE_RSVD_ONLY=1 timeout -k 10 200 python tools/pod_probe.py > $O/pod_probe.json || exit 1
cat $O/pod_probe.json
echo NEXTOK
