#!/bin/bash
# Paired pixel stores (VP8G_QPAIR=1 luma, 2 chroma, 3 both): quad tests on the "both" build, in-process
# A/B against the shipped build, then FETCH_SIZE / WRITE_SIZE of the bench kernel for each build.
set -o pipefail
L=webp-decoder_amd/lib
VP8G_LIB=$PWD/$L/ab/qpair3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_quad.py \
	-k "not stalled" > gpurun_out/qpair_tests.log 2>&1 || { tail -30 gpurun_out/qpair_tests.log; exit 1; }
tail -1 gpurun_out/qpair_tests.log
bash tools/gpu_abq.sh qpair ${RND:-4} $L/libvp8g.so $L/ab/qpair1.so $L/ab/qpair2.so $L/ab/qpair3.so || exit 1
export TMPDIR=/tmp
for v in base 3 1; do
	if [ $v = base ]; then export VP8G_LIB=$GRAFT_REPO_ROOT/$L/libvp8g.so; else export VP8G_LIB=$GRAFT_REPO_ROOT/$L/ab/qpair$v.so; fi
	for c in FETCH_SIZE WRITE_SIZE; do
		(cd /tmp && timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/qpair_pmc/$v/$c -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/qpair_pmc/$v.$c.log 2>&1) \
			|| { echo "pmc $v $c failed"; exit 1; }
	done
done
echo done
