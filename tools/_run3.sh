set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
: > $O/ring_sweep.txt
for sc in "office" "random_tris 1000000" "random_tris 300000"; do
  for r in 1 2; do
    for ring in 8 16; do
      echo "$sc ring=$ring $(RT_RING=$ring timeout -k 10 120 python tools/frame_probe.py $sc | tail -1)" >> $O/ring_sweep.txt || exit 1
    done
  done
done
cat $O/ring_sweep.txt
