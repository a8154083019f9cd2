#!/bin/bash
# Wide-tile slab stall hunt: the 2-rank rehearsal (W = 128) with A/B builds
# of the library (BURG_LIB).  BURG_SPIN_SECONDS=3: stalls fail fast.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-rehearse_ab4}
mkdir -p $O
cd $R
export BURG_SPIN_SECONDS=3
two() {
  name=$1; lib=$2; shift 2
  BURG_LIB=$R/finitedifference_amd/$lib timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) bench.py --gpus 2 --rehearse-one-gpu --steps 2 --warmup 1 "$@" > $O/$name.json 2> $O/$name.err
  echo "$name rc=$? $(grep -o '"value": [0-9.]*' $O/$name.json) $(grep -o 'rank[01]\]: finitedifference_amd._lib.BurgersError.*step/diagonal [0-9]*, wait 0x[0-9a-f]*' $O/$name.err | sed 's/finitedifference_amd._lib.BurgersError: libburgers_hip error -3: pipe engine: a wait timed out//' | tr '\n' ' ')"
}
two base libburgers_hip.so --nx 1024 --rows-per-gpu 1024 --stream-w 128
two nh1 libburgers_hip_nh1.so --nx 1024 --rows-per-gpu 1024 --stream-w 128
two nh2 libburgers_hip_nh2.so --nx 1024 --rows-per-gpu 1024 --stream-w 128
exit 0
