#!/bin/bash
# Ceiling of a read-back cut at 4096^2 (DESIGN.md
# section 9): throwaway builds whose loader skips the ring read-back of
# BURG_AB_SKIP diagonals of every W = 256 (WRONG results: the compute waves
# read stale window rows), all with the range check off (BURG_AB_NOCHECK:
# the fast path for every operand, so the stale values do not send the
# chains to the IEEE path) -- against the same build without the skip: the
# rate and the FETCH bytes a real cut of that share could reach at most.
# Two interleaved rounds per variant, then one FETCH_SIZE pass each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab_skip}; mkdir -p $O
B4="bench.py --steps 5 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check"
lib() { echo $PWD/finitedifference_amd/libburgers_hip_$1.so; }
V="nochk nochk_skip32 nochk_skip64 nochk_skip128"
for r in 1 2; do for v in $V; do
  BURG_LIB=$(lib $v) BURG_ALLOW_NONFINITE=1 timeout -k 10 200 python3 $B4 > $O/${v}_r$r.json 2> $O/${v}_r$r.err || { tail -5 $O/${v}_r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/${v}_r$r.json')); print('$v r$r', d['value'], d['roofline']['avg_launch_ms'], d['engine']['ieee_diagonals'])"
done; done
for v in $V; do
  BURG_LIB=$(lib $v) BURG_ALLOW_NONFINITE=1 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/${v}_FETCH_SIZE -o run -- python3 bench.py --steps 2 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check > /dev/null 2> $O/${v}_fetch.err || { tail -5 $O/${v}_fetch.err; exit 1; }
  echo "$v fetch ok"
done
echo ABOK
