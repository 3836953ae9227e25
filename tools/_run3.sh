set -o pipefail
export TMPDIR=/tmp
L=my-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "stack_ring or config4 or kat_scenes or adaptive_frames" > gpurun_out/t_ring.txt 2>&1 && tail -3 gpurun_out/t_ring.txt &&
timeout -k 10 900 python -u tools/ab_frame.py 2 $L/librt_hip_r02q.so $L/librt_hip_cur.so $L/librt_hip_deep.so -- random_tris 10000000 > gpurun_out/ab_rt.txt 2>&1 && tail -3 gpurun_out/ab_rt.txt &&
timeout -k 10 600 python -u tools/ab_frame.py 3 $L/librt_hip_cur.so $L/librt_hip_deep.so > gpurun_out/ab_off.txt 2>&1 && tail -2 gpurun_out/ab_off.txt
