#!/bin/bash
# Four-MB-rows-per-wave experiment (csrc/vp8g_quad.inc): digests and in-process A/B against the shipped
# build on uhd4, fhd4 and uhd4_yuv.  Usage: tools/gpu_quad.sh <tag> [rounds]
set -o pipefail
TAG=${1:-q}
RND=${2:-3}
OUT=gpurun_out/quad_$TAG
mkdir -p $OUT
for w in uhd4 fhd4 uhd4_yuv; do
	timeout -k 10 300 python3 -u tools/ab_inproc.py --workload $w --rounds $RND --steps 6 \
		webp-decoder_amd/lib/libvp8g.so webp-decoder_amd/lib/diag/libvp8g_quad.so > $OUT/$w.json 2> $OUT/$w.err || { echo "FAIL $w"; tail -5 $OUT/$w.err; exit 1; }
	echo "== $w"; cat $OUT/$w.json
done
