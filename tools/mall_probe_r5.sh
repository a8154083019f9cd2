#!/bin/bash
# Round-5 A/B for DESIGN 9(1): does the previous-state
# re-read get cheaper when one grid state fits the 256 MB Infinity Cache?
# Same 1024-tile pipe plans, state 268 MB (4096^2 W=256, 8192x2048 W=256)
# against 134 MB (4096x2048 W=128, 2048x4096 W=128); one 500-step
# trajectory per step, HIP-event kernel time.  Then HBM FETCH/WRITE passes of
# the 134 MB shape.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-mall_r5}
mkdir -p $O
cd $R
X="--steps 4 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --no-e2e --stencil-nx 0 --no-residual-check"
for cfg in "4096:4096:256" "8192:2048:256" "4096:2048:128" "2048:4096:128" "4096:4096:128"; do
  IFS=: read nx rows w <<< "$cfg"
  timeout -k 10 200 python bench.py --nx $nx --rows-per-gpu $rows --stream-w $w $X > $O/b_${nx}_${rows}_${w}.json 2> $O/b_${nx}_${rows}_${w}.err || { tail -5 $O/b_${nx}_${rows}_${w}.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$O/b_${nx}_${rows}_${w}.json'));print('$cfg',d['value'],d['roofline']['avg_launch_ms'],d['engine']['tiles'])"
done
cd /tmp
C="$R/bench.py --nx 4096 --rows-per-gpu 2048 --stream-w 128 --steps 2 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --no-e2e --stencil-nx 0 --no-residual-check"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $O/half_$ctr -o run -- python3 $C > /dev/null 2> $O/half_$ctr.err || { tail -5 $O/half_$ctr.err; exit 1; }
  echo "$ctr ok"
done
echo MALLOK
