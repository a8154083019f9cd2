#!/bin/bash
# Round-5 stencil A/B at 8192^2: time (rocprofv3 kernel stats) and HBM fetch
# (FETCH_SIZE pass) of the residual / J.x kernels per variant
# (BURG_STENCIL bits: 1 XCD-aware block order, 2 next-row prefetch) and row
# height (BURG_STENCIL_ROWS).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-stencil_ab_r5}
mkdir -p $O
cd /tmp
for cfg in ${CFGS:-"0:0" "1:0" "0:32" "1:32" "1:64" "3:32"}; do
  v=${cfg%%:*}; rows=${cfg##*:}
  tag=v${v}_r${rows}
  mkdir -p $O/$tag
  export BURG_STENCIL=$v
  if [ "$rows" = 0 ]; then unset BURG_STENCIL_ROWS; else export BURG_STENCIL_ROWS=$rows; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag/stats -o run -- python3 $R/tools/stencil_probe.py 8192 20 > $O/$tag/probe.json 2> $O/$tag/stats.err || { tail -5 $O/$tag/stats.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/$tag/fetch -o run -- python3 $R/tools/stencil_probe.py 8192 5 > /dev/null 2> $O/$tag/fetch.err || { tail -5 $O/$tag/fetch.err; exit 1; }
  echo "$tag ok"
done
echo ABOK
