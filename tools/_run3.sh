set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=$PWD/my-raytracer_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "adaptive or fuzz_analytic" > $O/t_adapt.txt 2>&1 && tail -1 $O/t_adapt.txt || exit 1
for r in 1 2; do
for t in sel8 selb; do
  RTAMD_HIP_LIB=$L/librt_hip_$t.so timeout -k 10 300 python bench.py --adaptive --no-cpu-baseline --steps 107 --warmup 107 > $O/b_$t.json 2>&1 || exit 1
  echo "$t $(grep -h '^{' $O/b_$t.json | cut -c100-170)"
done
done
