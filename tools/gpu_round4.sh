#!/bin/bash
# Round-4 bench pass (under gpurun): smoke, the default bench line, the N = 2
# rehearsals (per_gpu_alone; a device-ring failure on ALL ranks; ONE rank
# failing at its 4th launch), then the narrow-block A/B (A/B=1).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r4_round}
mkdir -p $O
cd $R
timeout -k 10 60 ./tools/probes/dma_high_probe > $O/dma_high_probe.txt 2>&1 || { cat $O/dma_high_probe.txt; exit 1; }
cat $O/dma_high_probe.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --rehearse-one-gpu --nx 8192 --rows-per-gpu 256 --stream-w 128 --steps 5 --warmup 1 > $O/bench_rehearse_n2.json 2> $O/bench_rehearse.err || { tail -20 $O/bench_rehearse.err; exit 1; }
cat $O/bench_rehearse_n2.json
BURG_TEST_FAIL_DEVICE_HALO=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --rehearse-one-gpu --nx 2048 --rows-per-gpu 1024 --stream-w 128 --steps 5 --warmup 1 --no-alone > $O/bench_rehearse_fallback.json 2> $O/bench_rehearse_fallback.err || { tail -20 $O/bench_rehearse_fallback.err; exit 1; }
grep '"halo_fallback": "device' $O/bench_rehearse_fallback.json > /dev/null || { echo "no fall-back recorded"; exit 1; }
# ONE rank (rank 1) fails at its launch number 3 (0-based: warm-up 0, timed 1, 2, 3 ...);
# rank 0's bounded waits must give up by themselves and every rank fall back together
BURG_SPIN_SECONDS=3 BURG_TEST_FAIL_DEVICE_HALO=1:3 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --rehearse-one-gpu --nx 2048 --rows-per-gpu 1024 --stream-w 128 --steps 5 --warmup 1 --no-alone > $O/bench_rehearse_failone.json 2> $O/bench_rehearse_failone.err || { tail -20 $O/bench_rehearse_failone.err; exit 1; }
grep '"halo_fallback": "device' $O/bench_rehearse_failone.json > /dev/null || { echo "no fall-back recorded (fail-one)"; exit 1; }
grep -h "bench.py rank" $O/bench_rehearse_failone.err | head -4
[ -n "$NO_MALL" ] || TAG=${TAG:-r4_round}_mall bash tools/probes/mall_probe.sh || exit 1
if [ "$AB" = "1" ]; then
  TAG=${TAG:-r4_round}_ab TESTLIB=$TESTLIB LIBS="$LIBS" bash tools/probes/ab_both.sh || exit 1
fi
echo ALLOK
