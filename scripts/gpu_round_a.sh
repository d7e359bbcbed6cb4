# First half of the round's evidence: smoke, the -m gpu suite, the bench line (with cpu_baseline),
# rocprofv3 kernel stats, the bench's PMC traffic passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_check.sh || exit 1
bash scripts/gpu_profile_round.sh || exit 1
echo round-a-done
