#!/bin/bash
# Round-5 A/B of the paired-halves kernel: rates and SQ stall decomposition
# (one PMC pass, 8 SQ counters) of the 1024^2 trajectory + 9-mu sweep.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-pair_ab}
mkdir -p $O
cd $R
for p in 0 1 0 1; do
  BURG_PAIR=$p timeout -k 10 120 python tools/probes/pair_ab.py 3 >> $O/rates.jsonl 2>> $O/rates.err || { tail -5 $O/rates.err; exit 1; }
done
cat $O/rates.jsonl
[ -n "$NO_SQ" ] && { echo PAIRABOK; exit 0; }
cd /tmp
for p in 0 1; do
  BURG_PAIR=$p timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $O/sq_p$p -o run -- python3 $R/tools/probes/pair_ab.py 1 > /dev/null 2> $O/sq_p$p.err || { tail -5 $O/sq_p$p.err; exit 1; }
  echo "sq p$p ok"
done
echo PAIRABOK
