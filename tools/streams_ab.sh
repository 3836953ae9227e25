#!/bin/bash
# Interleaved A/B of kernel libraries over launch shapes (frames per launch x launches in flight),
# bench.py medians per shape (dev tool, under gpurun).   usage: tools/streams_ab.sh ROUNDS lib1 lib2 ...
R=$1; shift
RAW=gpurun_out/streams_ab_raw.txt
mkdir -p gpurun_out; : > $RAW
SHAPES=("base20|--steps 20 --warmup 5" "f1s1|--frames 1 --streams 1 --steps 100 --warmup 20"
        "f1s3|--frames 1 --streams 3 --steps 100 --warmup 20" "f20s2|--frames 20 --streams 2 --steps 40 --warmup 20")
for r in $(seq 1 $R); do
  for sh in "${SHAPES[@]}"; do
    tag=${sh%%|*}; args=${sh#*|}
    for l in "$@"; do
      v=$(RTAMD_HIP_LIB=$l timeout -k 10 200 python bench.py $args --no-cpu-baseline --tree-record off --single-frames 0 2>/dev/null \
          | python -c "import json,sys; print(json.load(sys.stdin)['ms_per_step'])") || exit 1
      echo "$tag $(basename $l) $v" | tee -a $RAW
    done
  done
done
python - <<PY
import collections, statistics
d = collections.defaultdict(list)
for line in open("$RAW"):
    t, l, v = line.split(); d[(t, l)].append(float(v))
for (t, l), v in sorted(d.items()):
    print(f"{t:7s} {l:28s} median {statistics.median(v):.4f} ms/frame  ({min(v):.4f}-{max(v):.4f})")
PY
