#!/bin/bash
# A/B of the kept HALF block (BURG_KEEP_BLOCK=2: 8 of 16 diagonals in VGPRs, libburgers_hip_keep2.so,
# DESIGN.md section 4.1h): the wide-tile bitwise tests on the variant, then
# the 4096^2 headline interleaved base / keep (3 rounds) and one FETCH_SIZE
# pass each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab_keep}; mkdir -p $O
KL=$PWD/finitedifference_amd/libburgers_hip_keep2.so
BURG_LIB=$KL timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "wide or 4096 or 8192 or retained or slab_wide or steady_blocks or reserve or trajectory_from_initial or n8_slab" > $O/pytest_keep.log 2>&1 || { tail -30 $O/pytest_keep.log; exit 1; }
tail -1 $O/pytest_keep.log
B4="bench.py --steps 5 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e"
for r in 1 2 3; do for v in base keep2; do
  L=$PWD/finitedifference_amd/libburgers_hip.so; [ $v = keep2 ] && L=$KL
  BURG_LIB=$L timeout -k 10 200 python3 $B4 > $O/${v}_r$r.json 2> $O/${v}_r$r.err || { tail -5 $O/${v}_r$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${v}_r$r.json')); print('$v r$r', d['value'], d['roofline']['avg_launch_ms'], d['engine']['ieee_diagonals'], d['residual_check']['ok'])"
done; done
for v in base keep2; do
  L=$PWD/finitedifference_amd/libburgers_hip.so; [ $v = keep2 ] && L=$KL
  BURG_LIB=$L timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/${v}_FETCH_SIZE -o run -- python3 bench.py --steps 2 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check > /dev/null 2> $O/${v}_fetch.err || { tail -5 $O/${v}_fetch.err; exit 1; }
  echo "$v fetch ok"
done
echo ABOK
