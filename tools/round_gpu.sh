#!/bin/bash
# One GPU call of round evidence: the GPU test suite, the default bench line, the rocprofv3
# kernel-trace + HBM PMC passes (tools/profile_round.sh).  Usage on the box: bash tools/round_gpu.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/tests_$TAG.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed rc=$?"; exit 1; }
bash tools/profile_round.sh $TAG || exit 1
echo round_done
