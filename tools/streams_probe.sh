set -e
mkdir -p gpurun_out/r05zv
B="python -u bench.py --no-cpu-baseline --tree-record off --single-frames 0"
run() { tag=$1; shift; timeout -k 10 240 $B "$@" > gpurun_out/r05zv/$tag.json 2> gpurun_out/r05zv/$tag.err; echo "$tag $(python -c "import json,sys;d=json.load(open('gpurun_out/r05zv/$tag.json'));print(d['value'],d['ms_per_step'],d.get('frames_per_launch'))")"; }
run base20 --steps 20 --warmup 5
run f1s1 --frames 1 --streams 1 --steps 100 --warmup 20
run f1s2 --frames 1 --streams 2 --steps 100 --warmup 20
run f1s3 --frames 1 --streams 3 --steps 100 --warmup 20
run f10s2 --frames 10 --streams 2 --steps 20 --warmup 10
run f5s2 --frames 5 --streams 2 --steps 20 --warmup 10
run f20s2 --frames 20 --streams 2 --steps 40 --warmup 20
run base20b --steps 20 --warmup 5
