#!/bin/bash
# Non-temporal row loads for K1 / K2 (BURG_STENCIL bit 8): parity, then time / fetch
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-stencil_nt_r5}
mkdir -p $O
cd $R
for v in 8 10; do
  BURG_STENCIL=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "residual or jvp or stencils" > $O/pytest_v$v.log 2>&1 || { tail -20 $O/pytest_v$v.log; exit 1; }
done
echo parity ok
for r in 1 2; do CFGS="0:0 8:0 10:0" TAG=${TAG:-stencil_nt_r5}/round$r bash tools/stencil_ab_r5.sh || exit 1; done
