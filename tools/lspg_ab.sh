#!/bin/bash
# LSPG Gram kernel A/B on one box: parity tests, then the 1024^2 and 250^2
# probes with the warp-specialised Gram kernel (4 or 8 fill waves,
# BURG_LSPG_FILL_WAVES) and the one-role kernel (BURG_LSPG_GRAM=split).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-lspg_ab}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lspg" > $O/pytest_lspg.log 2>&1 || { tail -30 $O/pytest_lspg.log; exit 1; }
tail -2 $O/pytest_lspg.log
BURG_LSPG_FILL_WAVES=4 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lspg" > $O/pytest_lspg_fw4.log 2>&1 || { tail -30 $O/pytest_lspg_fw4.log; exit 1; }
tail -2 $O/pytest_lspg_fw4.log
for v in ws4 ws8 split; do
  G=ws; [ $v = split ] && G=split
  FW=4; [ $v = ws8 ] && FW=8
  for N in 1024 250; do
    BURG_LSPG_GRAM=$G BURG_LSPG_FILL_WAVES=$FW timeout -k 10 200 python tools/lspg_probe.py $N 95 10 > $O/probe_${N}_$v.json 2> $O/probe_$v.err || { tail -20 $O/probe_$v.err; exit 1; }
    python -c "import json; d=json.load(open('$O/probe_${N}_$v.json')); print('$v $N', {k: round(d[k],4) for k in ('ms_per_step','gram_ms_per_launch','gram_frac_hbm')}, d['its_per_step'][:4])"
  done
done
