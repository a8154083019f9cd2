#!/bin/bash
# Round-4 GPU pass (under gpurun): selected GPU tests (PYTEST_K), then
# optionally the default bench line (BENCH=1) and extra bench args (BENCH_ARGS).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r4}
mkdir -p $O
cd $R
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "$PYTEST_K" > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
  grep -E "PASSED|FAILED|ERROR|Gcell|passed|failed" $O/pytest_gpu.log | tail -40
fi
if [ "$BENCH" = "1" ]; then
  timeout -k 10 400 python bench.py $BENCH_ARGS > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
echo ALLOK
