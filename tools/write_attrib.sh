#!/bin/bash
# Write attribution (dev tool, under gpurun): HBM writes per frame (rocprofv3 WRITE_SIZE of the
# production render kernel, tools/pmc_summary.py with the committed calibration) of bench.py for
# kernel libraries that each drop one writer (measurement builds, make variant V=-DRT_MEAS_*):
#   RT_MEAS_NO_IMAGE   no image stores            RT_MEAS_NO_PSTATE  no path-state stores (colours only)
#   (round 5 also had RT_MEAS_NO_SUSP, for the suspend/resume variant removed since)
# usage: tools/write_attrib.sh TAG "bench args" lib1.so[#opt=v,...] lib2.so ...
set -e -o pipefail
TAG=${1:?tag}; ARGS=$2; shift 2
O=gpurun_out
export TMPDIR=/tmp
mkdir -p $O
for spec in "$@"; do
  l=${spec%%#*}
  opts=""
  name=$(basename $l .so)
  if [ "$spec" != "$l" ]; then
    for kv in $(echo ${spec#*#} | tr ',' ' '); do opts="$opts --opt $kv"; done
    name=${name}_$(echo ${spec#*#} | tr ',=' '__')
  fi
  B="python bench.py --no-cpu-baseline --tree-record off --single-frames 0 $ARGS $opts"
  RTAMD_HIP_LIB=$PWD/$l timeout -k 10 300 $B > $O/wa_${TAG}_$name.json
  RTAMD_HIP_LIB=$PWD/$l timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wa_${TAG}_${name}_w \
    -o run -- $B > $O/wa_${TAG}_${name}_w.log 2>&1
  python tools/pmc_summary.py $O/wa_${TAG}_$name.pmc.json --bench $O/wa_${TAG}_$name.json \
    --calib profiles/r02/hbm_calib.json $O/wa_${TAG}_${name}_w > /dev/null
  python -c "
import json; d = json.load(open('$O/wa_${TAG}_$name.pmc.json'))
b = json.loads(open('$O/wa_${TAG}_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['_per_frame']['hbm_write_bytes'] / 1e6, 2), 'MB/frame written,',
      b['value'], 'Mrays/s, frames/launch', b['config']['frames_per_launch'])" | tee -a $O/wa_${TAG}.txt
done
