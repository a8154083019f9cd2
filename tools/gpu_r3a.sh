#!/bin/bash
# Round-3 first GPU pass: the bench-regime parity tests, the slab residual /
# failed-context tests, a short headline bench with its residual check, and
# the N = 2 rehearsal (8192-wide slabs, label + residual check + fall-back).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r03a}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_regime.py -x -v --timeout 300 --timeout-method thread > $O/pytest_regime.log 2>&1 || { tail -40 $O/pytest_regime.log; exit 1; }
tail -3 $O/pytest_regime.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --rehearse-one-gpu --nx 8192 --rows-per-gpu 256 --stream-w 128 --steps 5 --warmup 1 > $O/bench_rehearse_n2.json 2> $O/bench_rehearse.err || { tail -20 $O/bench_rehearse.err; exit 1; }
cat $O/bench_rehearse_n2.json
BURG_TEST_FAIL_DEVICE_HALO=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --rehearse-one-gpu --nx 2048 --rows-per-gpu 1024 --stream-w 128 --steps 5 --warmup 1 > $O/bench_rehearse_fallback.json 2> $O/bench_rehearse_fallback.err || { tail -20 $O/bench_rehearse_fallback.err; exit 1; }
grep '"halo_fallback": "device' $O/bench_rehearse_fallback.json > /dev/null || { echo "no fall-back recorded"; exit 1; }
echo ALLOK
