#!/bin/bash
# LSPG PROM on the GPU box: parity tests, timing probes at 250^2 and 1024^2
# (npod 95, the reference driver's size), rocprofv3 kernel stats of the 1024^2 probe.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-lspg}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "lspg or ecsw or smoke" > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 200 python tools/lspg_probe.py 250 95 20 > $O/probe_250.json 2> $O/probe_250.err || { tail -20 $O/probe_250.err; exit 1; }
cat $O/probe_250.json
timeout -k 10 300 python tools/lspg_probe.py 1024 95 10 > $O/probe_1024.json 2> $O/probe_1024.err || { tail -20 $O/probe_1024.err; exit 1; }
cat $O/probe_1024.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/lspg_probe.py 1024 95 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
head -12 $O/prof/run_kernel_stats.csv
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/tools/lspg_probe.py 1024 95 3 > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/tools/lspg_probe.py 1024 95 3 > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 1; }
echo ALLOK
