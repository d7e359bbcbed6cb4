# GPU-box evidence for profiles/: the bench line, a rocprofv3 kernel-trace summary of the same
# command, and the two PMC passes (FETCH_SIZE / WRITE_SIZE, kernel-trace only) for roofline.traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/round
echo "== bench"; timeout -k 10 400 python bench.py > gpurun_out/round/bench.log 2>&1 || { tail -5 gpurun_out/round/bench.log; exit 1; }
tail -1 gpurun_out/round/bench.log
B="python bench.py --no-cpu-baseline"
echo "== stats"; timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/round/prof -o bench -- $B > gpurun_out/round/prof.log 2>&1 || exit 1
echo "== fetch"; timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/round/pmc/fetch -o run -- $B > gpurun_out/round/fetch.log 2>&1 || exit 1
echo "== write"; timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/round/pmc/write -o run -- $B > gpurun_out/round/write.log 2>&1 || exit 1
echo done
