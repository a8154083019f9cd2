#!/bin/bash
# A/B of the comm wave's poll window for blocks of 16 (BURG_U16_LA: 32
# default, 48, 64) on the N = 8 per-GPU slab (16384 x 2048, W = 512) and on
# 4096^2 (W = 256), two rounds each
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_la}
mkdir -p $O
rm -f $O/ab.txt
X="--no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check --steps 3 --warmup 1"
for rep in 1 2; do
for lib in libburgers_hip.so libburgers_hip_la48.so libburgers_hip_la64.so; do
  BURG_LIB=finitedifference_amd/$lib timeout -k 10 200 python bench.py --nx 16384 --rows-per-gpu 2048 $X > $O/s.json 2> $O/s.err || { tail -5 $O/s.err; exit 1; }
  python -c "import json; d=json.load(open('$O/s.json')); print('$lib 16384x2048', d['value'], d['ms_per_step'], d['engine']['blocked_diagonals'])" >> $O/ab.txt
  BURG_LIB=finitedifference_amd/$lib timeout -k 10 200 python bench.py $X > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$lib 4096x4096', d['value'], d['ms_per_step'], d['engine']['blocked_diagonals'])" >> $O/ab.txt
done
done
cat $O/ab.txt
echo ABOK
