set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=$PWD/my-raytracer_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "adaptive or fuzz_analytic" > $O/t_adapt.txt 2>&1 && tail -1 $O/t_adapt.txt || exit 1
for t in 2 8; do
  RTAMD_HIP_LIB=$L/librt_hip_row$t.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sel$t -o run -- python bench.py --adaptive --no-cpu-baseline --steps 32 --warmup 32 > $O/prof_sel$t.log 2>&1 || exit 1
  echo "sel$t $(grep -h '^{' $O/prof_sel$t.log | cut -c100-200) $(grep -h select $O/prof_sel$t/run_kernel_stats.csv | cut -d, -f12-16)"
done
