#!/bin/bash
# Round-5 baseline on the GPU: the default bench line, rocprofv3 kernel stats of
# the headline trajectory, and fresh K1 / K2 stencil HBM passes at 8192^2
# (the round-1 counters predate the stencil rework).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r5base}
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench ok
HEAD="bench.py --steps 10 --warmup 2 --no-1024 --no-rom --no-cpu-baseline --no-e2e --stencil-nx 0 --no-residual-check"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_head -o run -- python3 $R/$HEAD > $O/prof_head.json 2> $O/prof_head.err || { tail -20 $O/prof_head.err; exit 1; }
echo head stats ok
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stencil -o run -- python3 $R/tools/stencil_probe.py 8192 20 > $O/prof_stencil.log 2>&1 || { tail -20 $O/prof_stencil.log; exit 1; }
echo stencil stats ok
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_stencil -o run -- python3 $R/tools/stencil_probe.py 8192 5 > $O/pmc_fetch_stencil.log 2>&1 || { tail -20 $O/pmc_fetch_stencil.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_stencil -o run -- python3 $R/tools/stencil_probe.py 8192 5 > $O/pmc_write_stencil.log 2>&1 || { tail -20 $O/pmc_write_stencil.log; exit 1; }
echo ALLOK
