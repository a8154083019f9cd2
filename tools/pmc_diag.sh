#!/bin/bash
# SQ/GRBM stall breakdown of the bench's march kernel (diagnostics), one
# rocprofv3 pass per counter set (MI355X_MICROARCH.md: <= 8 SQ, 2 GRBM).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-diag}
mkdir -p $O
cd /tmp
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline}
n=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $O/pmc$n -o run -- python3 $R/bench.py $ARGS > $O/pmc$n.log 2>&1 || { tail -5 $O/pmc$n.log; exit 1; }
done
echo ALLOK
