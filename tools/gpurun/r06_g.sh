# usage: bash tools/gpurun/r06_g.sh TAG -- scheduler-variant A/B of the hash TUs (r06_f.sh: base, noilp, mix), then
# three interleaved rounds of spec_large on / off on C5, C1 and C4 (r06_e.sh, rounds cut to 3)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
bash tools/gpurun/r06_f.sh ${TAG}v base noilp mix
bash tools/gpurun/r06_e.sh ${TAG}s
