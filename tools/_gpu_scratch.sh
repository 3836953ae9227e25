set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export CALIB=profiles/r02/hbm_calib.json
bash tools/configs_bench.sh r03z || exit 1
bash tools/profile_round.sh rt10m_r03z --scene random_tris --tris 10000000 || exit 1
