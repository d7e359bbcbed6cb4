# Round 3 diagnostic: per-Gaussian pair counts of two depth-sort variants (scripts/dsort_diag2.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
for L in libgs_base.so libgs_mi355x.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python scripts/dsort_diag2.py 3500000 || exit 1
done
