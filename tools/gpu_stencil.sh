#!/bin/bash
# GPU pass for the stencil rewrite: parity tests, bench, stencil rocprof.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-stencil}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stencil -o run -- python3 $R/tools/stencil_probe.py 8192 20 > $O/prof_stencil.log 2>&1 || { tail -20 $O/prof_stencil.log; exit 1; }
tail -2 $O/prof_stencil.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_stencil -o run -- python3 $R/tools/stencil_probe.py 8192 5 > $O/pmc_fetch_stencil.log 2>&1 || { tail -20 $O/pmc_fetch_stencil.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_stencil -o run -- python3 $R/tools/stencil_probe.py 8192 5 > $O/pmc_write_stencil.log 2>&1 || { tail -20 $O/pmc_write_stencil.log; exit 1; }
echo ALLOK
