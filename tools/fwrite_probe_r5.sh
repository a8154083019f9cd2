set -o pipefail
O=gpurun_out/fwrite; mkdir -p $O
gcc -O2 -pthread -o $O/fwp tools/probes/file_write_probe.c || exit 1
for r in 1 2; do for m in 0 1; do for t in 1 2 4 8; do
  timeout -k 5 60 $O/fwp /tmp/fwp_$$.bin $t $m 8192 >> $O/rates.txt || exit 1
done; done; done
df -h /tmp >> $O/rates.txt; mount | grep -E " / | /tmp " >> $O/rates.txt || true
