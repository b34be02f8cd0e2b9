# round 2 closing evidence after the lane-kernel changes: part A (suite, smoke, bench lines),
# then rocprofv3 stats + FETCH/WRITE passes of the lane configs (the wave kernel is unchanged)
set -o pipefail
bash tools/r2_round.sh || exit $?
for c in c4 c5 c2_big; do bash tools/profile_round.sh $c || exit 3; done
PROF_NAME=c4_8192 bash tools/profile_round.sh c4 --batch 8192 || exit 4
