set -o pipefail
export TMPDIR=/tmp
L=my-raytracer_amd/lib/variants
timeout -k 10 600 python -u tools/ab_frame.py 4 $L/librt_hip_base.so $L/librt_hip_cur.so > gpurun_out/ab.txt 2>&1; tail -2 gpurun_out/ab.txt
