#!/bin/bash
# residual's per-block sum of squares: LDS tree (default) vs wave butterflies (sw)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sumsq_ab
mkdir -p $O
cd $R
[ -n "$SKIP_PARITY" ] || BURG_LIB=finitedifference_amd/libburgers_hip_sw.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_regime.py -k "residual or jvp or stencils" > $O/pytest_sw.log 2>&1 || { tail -20 $O/pytest_sw.log; exit 1; }
[ -n "$SKIP_PARITY" ] || tail -1 $O/pytest_sw.log
cd /tmp
for r in 1 2; do mkdir -p $O/r$r; for v in base sw; do
  if [ $v = sw ]; then L=$R/finitedifference_amd/libburgers_hip_sw.so; else L=$R/finitedifference_amd/libburgers_hip.so; fi
  BURG_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r$r/$v -o run -- python3 $R/tools/stencil_probe.py 8192 20 > $O/r$r/$v.json 2> $O/r$r/$v.err || { tail -5 $O/r$r/$v.err; exit 1; }
done; done
echo ABOK
