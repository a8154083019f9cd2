#!/bin/bash
# Round-6 checkpoint on a fresh box: the whole GPU suite, smoke, the default
# bench line, and the N = 2 rehearsal (two slab ranks sharing the one GPU:
# the N > 1 bench path with its per-rank diagnostics).
#   TAG=name [SKIP_SUITE=1] [SKIP_BENCH=1] bash tools/gpu_r6.sh
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r6check}
mkdir -p $O
cd $R
if [ -z "$SKIP_SUITE" ]; then
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench ok
fi
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29702 bench.py --gpus 2 --rehearse-one-gpu --nx 2048 --rows-per-gpu 512 --stream-w 128 --steps 5 --warmup 1 2> $O/n2.err | grep '^{' > $O/bench_rehearse_n2.json || { tail -5 $O/n2.err; exit 1; }
echo REHEARSE_OK
