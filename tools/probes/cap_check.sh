# capped trajectory ring in one launch: the regime tests, then the N = 8
# per-GPU slab (16384 x 2048: its ring is capped by free HBM) with its
# residual self-check
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-cap}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_regime.py -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -3 $O/t.log
X="--no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --steps 3 --warmup 1"
timeout -k 10 300 python bench.py --nx 16384 --rows-per-gpu 2048 $X > $O/s16.json 2> $O/s16.err || { tail -5 $O/s16.err; exit 1; }
python -c "import json; d=json.load(open('$O/s16.json')); print('16384x2048', d['value'], d['ms_per_step'], d['engine'], d['residual_check']['rel'], d['residual_check']['ok'])"
