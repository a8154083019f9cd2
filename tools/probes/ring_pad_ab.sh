#!/bin/bash
# A/B of the trajectory ring's per-tile stride (BURG_RING_PAD: 0 = none, unset = odd) at the
# bench shapes, plain and retained (snap_every=10) rings; two rounds.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-ring_pad}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for round in 1 2; do
  for pad in 0 odd 17; do
    for cfg in "4096 4096 1" "16384 2048 1" "16384 2048 10" "8192 2048 10"; do
      if [ "$pad" = odd ]; then unset BURG_RING_PAD; else export BURG_RING_PAD=$pad; fi
      timeout -k 10 120 python tools/probes/traj_rate.py $cfg 3 >> $O/rates.jsonl || exit 1
      tail -1 $O/rates.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('pad=$pad', d['grid'], 'k', d['snap_every'], d['gcell_per_s_best'], d['kernel_ms'])"
    done
  done
done
