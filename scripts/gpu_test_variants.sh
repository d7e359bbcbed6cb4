# parity tests (selected by PYTEST_K) for each library variant in $VARIANTS, no early exit on failure
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in ${VARIANTS:-mi355x}; do
  echo "== $v"
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 600 python -m pytest tests -m gpu -q -k "${PYTEST_K:-parity}" > gpurun_out/ab/pytest_$v.log 2>&1
  rc=$?
  tail -3 gpurun_out/ab/pytest_$v.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo done
