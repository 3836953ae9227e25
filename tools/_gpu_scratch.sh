set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u tools/diag_probe.py office > $O/r03zc_diag_office.txt 2>&1 || { tail $O/r03zc_diag_office.txt; exit 1; }
timeout -k 10 300 python -u tools/diag_probe.py random_tris 1920 1080 1 10000000 > $O/r03zc_diag_rt10m.txt 2>&1 || { tail $O/r03zc_diag_rt10m.txt; exit 1; }
cat $O/r03zc_diag_office.txt $O/r03zc_diag_rt10m.txt
