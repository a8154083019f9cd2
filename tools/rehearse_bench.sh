#!/bin/bash
# The N > 1 bench path (slab contexts, device-ring halo with its self-test,
# reserve before the barrier, max-over-ranks timing) rehearsed with 2, 3 and
# 4 ranks sharing the one-GPU box (gloo; 2048 x 512 per rank at W = 128, so
# every rank's workgroups are resident together).  Ranks share one GPU, so
# the values say nothing about scaling -- they check that the path runs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-rehearse_bench}
mkdir -p $O
cd $R
for n in 2 3 4; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus $n --rehearse-one-gpu --nx 2048 --rows-per-gpu 512 --stream-w 128 --steps 5 --warmup 1 2>$O/n$n.err | grep '^{' > $O/bench_rehearse_n$n.json || { tail -5 $O/n$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_rehearse_n$n.json')); print($n, d['value'], d['ms_per_step'], d['config']['halo_ring'])"
done
