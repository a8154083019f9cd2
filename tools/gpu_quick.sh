#!/bin/bash
# Quick GPU pass (under gpurun): GPU parity tests, default bench, and the
# larger BASELINE configs as timing probes (config 2: 4096^2).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-quick}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
for T in ${BIG_T:-100}; do
timeout -k 10 200 python bench.py --nx 4096 --time-steps $T --steps 2 --warmup 1 --no-cpu-baseline > $O/bench4096_T$T.json 2> $O/bench4096.err || { tail -20 $O/bench4096.err; exit 1; }
cat $O/bench4096_T$T.json
done
echo ALLOK
