#!/bin/bash
# rocprofv3 passes of the default bench (4096^2 trajectory) under gpurun:
# kernel stats, HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes), and
# two SQ passes (issue / wait breakdown of the pipe kernel).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-prof}
mkdir -p $O
cd $R
B="bench.py --steps ${STEPS:-3} --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 ${EXTRA}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $B > $O/bench_stats.json 2> $O/stats.err || { tail -5 $O/stats.err; exit 1; }
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $B > /dev/null 2> $O/fetch.err || { tail -5 $O/fetch.err; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $B > /dev/null 2> $O/write.err || { tail -5 $O/write.err; exit 1; }
if [ -n "$SQ" ]; then
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $O/sq1 -o run -- python3 $B > /dev/null 2> $O/sq1.err || { tail -5 $O/sq1.err; exit 1; }
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/sq2 -o run -- python3 $B > /dev/null 2> $O/sq2.err || { tail -5 $O/sq2.err; exit 1; }
fi
cat $O/bench_stats.json
find $O -name "*kernel_stats.csv" | head -3
echo PROFOK
