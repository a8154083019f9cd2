#!/bin/bash
# A/B of the K1/K2 stencil variants (BURG_STENCIL bits: 1 XCD-aware block
# order, 2 next-row prefetch, 4 two columns per thread) at 8192^2, two rounds,
# one line per variant (VARIANTS: the list).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-stencil_ab}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for round in 1 2; do
  for v in ${VARIANTS:-0 1 2 3}; do
    BURG_STENCIL=$v timeout -k 10 120 python tools/stencil_probe.py ${NX:-8192} 50 > $O/v${v}_r${round}.json || exit 1
    echo "v$v r$round $(python -c "import json,sys; d=json.load(open('$O/v${v}_r${round}.json')); print(d['residual']['avg_launch_ms'], d['residual']['frac'], d['jvp']['avg_launch_ms'], d['jvp']['frac'])")"
  done
done
