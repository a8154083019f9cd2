set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/d1
cd $R
BURG_STREAM_DEBUG=8 timeout -k 10 120 python tools/prof_stream.py 1024 500 > gpurun_out/d1/why500.log 2>&1 || exit 1
BURG_STREAM_DEBUG=8 timeout -k 10 120 python tools/prof_stream.py 1024 50 > gpurun_out/d1/why50.log 2>&1 || exit 1
timeout -k 10 200 python tools/stream_rate.py > gpurun_out/d1/rate.log 2>&1 || exit 1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/d1/prof -o run -- python3 $R/bench.py --steps 500 --no-cpu-baseline > $R/gpurun_out/d1/prof.log 2>&1 || exit 1
n=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_VMEM_WR" "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/gpurun_out/d1/pmc$n -o run -- python3 $R/tools/prof_stream.py 1024 500 > $R/gpurun_out/d1/pmc$n.log 2>&1 || exit 1
done
echo ok
