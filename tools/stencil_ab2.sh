#!/bin/bash
# A/B of the K1/K2 stencils' block height (BURG_STENCIL_ROWS) and the fused
# norm sum (BURG_SUMSQ_FUSED) at 8192^2; two rounds; the bitwise stencil tests
# first with the defaults.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-stencil_ab2}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "stencil or residual or jvp or newton" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for round in 1 2; do
  for cfg in ${CFGS:-"64 0" "64 1" "32 0" "32 1" "16 0" "16 1"}; do
    set -- $cfg
    BURG_STENCIL_ROWS=$1 BURG_SUMSQ_FUSED=$2 timeout -k 10 120 python tools/stencil_probe.py ${NX:-8192} 50 > $O/rows$1_f$2_r$round.json || exit 1
    echo "rows=$1 fused=$2 r$round $(python -c "import json; d=json.load(open('$O/rows$1_f$2_r$round.json')); print(d['residual']['avg_launch_ms'], d['residual']['frac'], d['jvp']['avg_launch_ms'], d['jvp']['frac'])")"
  done
done
