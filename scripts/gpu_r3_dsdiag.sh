# Round 3 diagnostic: depth sort variants at growing N (scripts/dsort_diag.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
for L in libgs_mi355x.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python scripts/dsort_diag.py 3500000 5000000 || exit 1
done
