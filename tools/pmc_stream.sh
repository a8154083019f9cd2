#!/bin/bash
# PMC passes over one streaming advance (diagnostics): run on the GPU box.
set -e
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; cd /tmp
O=$R/gpurun_out/pmc
mkdir -p $O
for flags in 0 1; do
  export BURG_STREAM_DEBUG=$flags
  n=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU" \
             "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_BUSY_CYCLES" \
             "GRBM_GUI_ACTIVE SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE"; do
    n=$((n+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set -d $O/f${flags}_p$n -o run -- python3 $R/tools/prof_stream.py > $O/f${flags}_p$n.log 2>&1
  done
done
echo done
