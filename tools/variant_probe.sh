#!/bin/bash
# times the production kernel for each library variant in lib/variants (dev tool)
for lib in my-raytracer_amd/lib/librt_hip.so my-raytracer_amd/lib/variants/*.so; do
  echo "== $lib"
  RTAMD_HIP_LIB=$lib timeout -k 10 300 python tools/perf_probe.py ${@:-quick} 2>&1 | grep -v amdgpu.ids
done
