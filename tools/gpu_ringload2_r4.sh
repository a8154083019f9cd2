#!/bin/bash
# ring_load with coalesced reads: the trajectory / sweep / retained tests, then
# kernel stats of a short 4096^2 bench run
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r4rl2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "pipe or traj or retained or sweep or regime or parity" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 5 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check > $O/bench.json 2> $O/stats.err || { tail -5 $O/stats.err; exit 1; }
cat $O/bench.json
echo NEXTOK
