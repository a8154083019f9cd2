#!/bin/bash
# Full GPU pass (under gpurun): every GPU test, smoke, default bench, the LSPG
# and snapshot-I/O probes.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-round}
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
# the N > 1 bench path (slab contexts, halo self-test, max-over-ranks timing)
# rehearsed with 2 ranks sharing the box's GPU (gloo; W = 128 so both slabs'
# workgroups are resident together)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --rehearse-one-gpu --nx 8192 --rows-per-gpu 256 --stream-w 128 --steps 5 --warmup 1 > $O/bench_rehearse_n2.json 2> $O/bench_rehearse.err || { tail -20 $O/bench_rehearse.err; exit 1; }
cat $O/bench_rehearse_n2.json
# the same with every device-ring launch failing (test hook): the bench must
# fall back to the host rings on all ranks and still print its line
BURG_TEST_FAIL_DEVICE_HALO=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --rehearse-one-gpu --nx 2048 --rows-per-gpu 1024 --stream-w 128 --steps 5 --warmup 1 > $O/bench_rehearse_fallback.json 2> $O/bench_rehearse_fallback.err || { tail -20 $O/bench_rehearse_fallback.err; exit 1; }
grep '"halo_fallback": "device' $O/bench_rehearse_fallback.json > /dev/null || { echo "no fall-back recorded"; exit 1; }
timeout -k 10 300 python tools/snapio_probe.py 1024 100 /tmp/snapio > $O/snapio_1024.json 2> $O/snapio.err || { tail -20 $O/snapio.err; exit 1; }
cat $O/snapio_1024.json
echo ALLOK
