# One box: config-5 A/B (ab_cfg5.sh) then a bench A/B (ab.sh); variables as in those scripts
# (V5 / VB: the variants of each half).
set -o pipefail
cd $GRAFT_REPO_ROOT
VARIANTS="$V5" REPS=${REPS5:-2} TESTS=$TESTS PYTEST_K="$PYTEST_K" bash scripts/ab_cfg5.sh || exit 1
VARIANTS="$VB" REPS=${REPSB:-3} TESTS= bash scripts/ab.sh || exit 1
echo combo-done
