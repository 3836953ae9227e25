set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
L=$PWD/my-raytracer_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "frames or stripes or full_size_office" > $O/t_band.txt 2>&1 && tail -1 $O/t_band.txt || exit 1
for r in 1 2; do
for v in noband band; do
  RTAMD_HIP_LIB=$L/librt_hip_$v.so timeout -k 10 300 python bench.py --width 3840 --height 2160 --spp 4 --steps 16 --warmup 4 --single-frames 0 --no-cpu-baseline > $O/c3_$v.json 2>/dev/null || exit 1
  RTAMD_HIP_LIB=$L/librt_hip_$v.so timeout -k 10 300 python bench.py --steps 256 --warmup 128 --single-frames 0 --no-cpu-baseline > $O/c2_$v.json 2>/dev/null || exit 1
  RTAMD_HIP_LIB=$L/librt_hip_$v.so timeout -k 10 300 python bench.py --scene random_tris --tris 10000000 --steps 64 --warmup 16 --single-frames 0 --no-cpu-baseline > $O/c4_$v.json 2>/dev/null || exit 1
  echo "$r $v $(python -c "
import json
for c in ('c2','c3','c4'):
    d=json.loads(open('$O/'+c+'_$v.json').read().strip().splitlines()[-1]); print(c, d['value'], d['ms_per_step'], end='  ')
")"
done
done
