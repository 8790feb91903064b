#!/bin/bash
# Round-3 evidence in one GPU call: extended VALU issue-cost microbenchmark, the GPU tests, the
# default bench line, rocprofv3 kernel trace + HBM passes (profile_round.sh) and the SQ instruction /
# wait / LDS-conflict PMC groups of the bench kernel (pmc_pass.sh).  Stops at the first failure.
#   bash tools/round3_gpu.sh <tag> [skip-tests]
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 200 tools/ubench/valu_rates2 > gpurun_out/valu_rates2_$TAG.txt 2>&1 || { echo "valu_rates2 failed rc=$?"; exit 1; }
echo ubench_done
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/tests_$TAG.log; exit 1; }
  tail -3 gpurun_out/tests_$TAG.log
fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed rc=$?"; exit 1; }
cat gpurun_out/bench_$TAG.json | cut -c1-400
bash tools/profile_round.sh $TAG || exit 1
bash tools/pmc_pass.sh gpurun_out/pmc_$TAG --no-cpu-baseline --e2e-frames 0 --extra none --encode none --steps 2 --warmup 1 || exit 1
echo round_done
