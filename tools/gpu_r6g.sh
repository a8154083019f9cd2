#!/bin/bash
# Round-6 closing check of the final sources on a fresh box: the whole GPU
# suite, smoke, rocprofv3 kernel stats of the default bench command and the
# 4096^2 HBM / clock passes (tools/prof_r3.sh NAMES=b4), the default bench
# line, the N = 2 rehearsal
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
TAG=prof_r6g NAMES="b4" bash tools/prof_r3.sh || exit 1
SKIP_SUITE=1 TAG=r6g bash tools/gpu_r6.sh || exit 1
