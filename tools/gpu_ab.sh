#!/bin/bash
# One GPU call: the GPU test suite (optional), then an interleaved in-process A/B of libvp8g builds
# on the bench workloads (tools/ab_inproc.py).  Outputs under gpurun_out/ab_<tag>/.
#   bash tools/gpu_ab.sh <tag> <tests:0|1> <workloads, e.g. uhd4,fhd4> lib1.so lib2.so ...
set -u
TAG=$1; TESTS=$2; WLS=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/ab_$TAG
mkdir -p "$O"
if [ "$TESTS" = 1 ]; then
	timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > "$O/tests.log" 2>&1 \
		|| { echo "tests failed rc=$?"; tail -40 "$O/tests.log"; exit 1; }
	tail -3 "$O/tests.log"
fi
for W in ${WLS//,/ }; do
	timeout -k 10 420 python -u tools/ab_inproc.py --workload "$W" --rounds 6 --steps 8 "$@" > "$O/$W.jsonl" 2> "$O/$W.err" \
		|| { echo "ab $W failed rc=$?"; tail -20 "$O/$W.err"; exit 1; }
	echo "== $W"; cat "$O/$W.jsonl"
done
echo ab_done
