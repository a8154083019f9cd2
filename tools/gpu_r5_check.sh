#!/bin/bash
# Round-5 checkpoint on a fresh box: the whole GPU suite, smoke, the default
# bench line, and the N = 8 per-GPU slab line (16384 x 2048, snap_every 10,
# one rank, no halo).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r5check}
mkdir -p $O
cd $R
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench ok
timeout -k 10 300 python bench.py --nx 16384 --rows-per-gpu 2048 --snap-every 10 --steps 3 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e > $O/slab_16384x2048.json 2> $O/slab.err || { tail -20 $O/slab.err; exit 1; }
echo BENCHES_OK
# N = 2 rehearsal: two slab ranks sharing the one GPU (the N > 1 bench path)
cd $R
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29702 bench.py --gpus 2 --rehearse-one-gpu --nx 2048 --rows-per-gpu 512 --stream-w 128 --steps 5 --warmup 1 2> $O/n2.err | grep '^{' > $O/bench_rehearse_n2.json || { tail -5 $O/n2.err; exit 1; }
echo REHEARSE_OK
