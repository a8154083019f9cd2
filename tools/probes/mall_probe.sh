#!/bin/bash
# Does a ring read-back that fits the 256 MB Infinity Cache run faster?  The
# trajectory rate at grids whose one-step state (16 B x cells) is below,
# near and above 256 MB, one process each (traj_rate.py, plain ring).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-mall}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for cfg in "4096 4096" "2048 4096" "4096 2048" "2048 2048" "8192 1024" "1024 8192"; do
  timeout -k 10 120 python tools/probes/traj_rate.py $cfg 1 3 >> $O/rates.jsonl || exit 1
  tail -1 $O/rates.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['grid'], 'W', d['W'], d['gcell_per_s_best'], d['kernel_ms'])"
done
