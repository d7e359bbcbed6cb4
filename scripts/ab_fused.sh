# The fused forward + backward prototype (gs_debug_set_fused_blend) against the default blends:
# its bit-identity test, then alternating bench runs of the HEAD library (cur), the working tree's
# default path (refac) and the working tree's fused path, and a kernel trace of the fused path.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/fz; mkdir -p $O; rm -rf $O/*
GS_MI355X_LIB=libgs_refac.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "fused_blend or graph_backwards or split" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in cur refac fused; do
    lib=$v; a=""; [ $v = fused ] && { lib=refac; a="--fused-blend"; }
    GS_MI355X_LIB=libgs_$lib.so timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline $a > $O/${v}_$r.log 2>&1 || { tail -3 $O/${v}_$r.log; exit 1; }
    python -c "import json;d=json.loads(open('$O/${v}_$r.log').read().strip().splitlines()[-1]);print('$v',$r,round(d['ms_per_step'],4),{k:round(x,4) for k,x in d['stage_ms'].items()})"
  done
done
GS_MI355X_LIB=libgs_refac.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --fused-blend > $O/prof.log 2>&1
echo prof rc=$?
