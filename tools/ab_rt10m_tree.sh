#!/bin/bash
# Config 4 (10 M random triangles) A/B of device-tree build options (dev tool, under gpurun):
# pixels are identical for any tree, so only time and traversal work change.
#   bash tools/ab_rt10m_tree.sh TAG "opt-set-1" "opt-set-2" ...   (an opt set: "k=v k=v" or "base")
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}; shift
O=gpurun_out/ab_$TAG
mkdir -p $O
i=0
for s in "$@"; do
  args=""
  [ "$s" != "base" ] && for kv in $s; do args="$args --opt $kv"; done
  timeout -k 10 300 python -u bench.py --scene random_tris --tris 10000000 --no-cpu-baseline --single-frames 0 $args \
    > $O/v$i.json 2> $O/v$i.err || { echo "variant $i ($s) failed"; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/v$i.json')); print('$s', d['value'], d['kernel_ms_per_frame'], d['config'].get('device_scene_MB'), d['config'].get('host_bvh_build_s'))" | tee -a $O/summary.txt
  i=$((i+1))
done
