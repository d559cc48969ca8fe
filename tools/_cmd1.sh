set -e
bash tools/prof_round.sh c2 c3 c5 c5p8 c2a c5a
