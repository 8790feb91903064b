#!/bin/bash
# Round-end GPU run: GPU tests, smoke, default bench, kernel-trace + traffic profile, device-m05
# kernel trace.  Usage (repo root, on the box): bash tools/final_run.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -20 $O/gpu_tests_$TAG.log; exit 1; }
tail -2 $O/gpu_tests_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke_$TAG.log; exit 1; }
tail -1 $O/smoke_$TAG.log
timeout -k 10 600 python -u bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo "bench failed rc=$?"; tail -20 $O/bench_$TAG.err; exit 1; }
bash tools/profile_round.sh $TAG || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG/m05 -o m05 -- \
  python3 $R/tools/m05_kernel_probe.py 0 1 1024 > $O/prof_$TAG/m05.log 2>&1 || { echo "m05 trace failed rc=$?"; exit 1; }
echo final_done
