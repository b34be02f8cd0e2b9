# round 2 evidence, part B: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes per config
set -o pipefail
for c in c2 c3 c4 c5 c2_big; do bash tools/profile_round.sh $c || exit 3; done
PROF_NAME=c4_8192 bash tools/profile_round.sh c4 --batch 8192 || exit 4
