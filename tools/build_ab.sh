#!/bin/bash
# Builds lib/variants/librt_hip_NAME.so from the kernel source of git revision REV (the current
# host objects), for interleaved A/B runs against the working tree (tools/ab.sh, ab_frame.py) --
# dev tool, CPU side.   usage: tools/build_ab.sh REV NAME [extra hipcc flags]
set -e
REV=${1:?rev}; NAME=${2:?name}; shift 2
cd "$(dirname "$0")/../my-raytracer_amd"
SRC=csrc/device/_ab_$NAME.hip
git show "$REV:my-raytracer_amd/csrc/device/rt_render.hip" > $SRC
make -s lib/device_image.o
make -s variant HIP_SRC=$SRC N=$NAME V="$*"
rm -f $SRC
ls -la lib/variants/librt_hip_$NAME.so
