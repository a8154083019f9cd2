#!/bin/bash
# Round-5 resident-layout stencils (BURG_STENCIL bit 4): parity under each
# variant, then the same time / FETCH_SIZE A/B as stencil_ab_r5.sh.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-stencil_res_r5}
mkdir -p $O
cd $R
for v in 4 5 7; do
  BURG_STENCIL=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "residual or jvp or stencils" > $O/pytest_v$v.log 2>&1 || { tail -20 $O/pytest_v$v.log; exit 1; }
done
echo parity ok
CFGS="0:0 4:0 5:0 6:0 7:0" TAG=${TAG:-stencil_res_r5} bash tools/stencil_ab_r5.sh
