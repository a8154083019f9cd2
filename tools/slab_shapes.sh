#!/bin/bash
# Per-GPU slab shapes of BASELINE configs[3] / configs[4] (8192- and
# 16384-wide rows, 2048 rows per GPU) and the 8192^2 single-GPU grid, each
# run as ONE rank on one GPU (bench.py, world 1): the per-GPU rate the weak
# scaling curve starts from.  Output: gpurun_out/${TAG}/slab_*.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-slabs}
mkdir -p $O
cd $R
X="--no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --steps 5 --warmup 1"
timeout -k 10 200 python bench.py --nx 8192 --rows-per-gpu 2048 $X > $O/slab_8192x2048.json 2> $O/slab_8192.err || { tail -20 $O/slab_8192.err; exit 1; }
timeout -k 10 200 python bench.py --nx 16384 --rows-per-gpu 2048 $X > $O/slab_16384x2048.json 2> $O/slab_16384.err || { tail -20 $O/slab_16384.err; exit 1; }
timeout -k 10 300 python bench.py --nx 8192 $X --steps 2 > $O/grid_8192x8192.json 2> $O/grid_8192.err || { tail -20 $O/grid_8192.err; exit 1; }
for f in $O/slab_*.json $O/grid_*.json; do python -c "
import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['engine'], d['roofline']['frac'], d.get('issue_roofline',{}).get('frac'))"; done
