#!/bin/bash
# In-process A/B of several builds on uhd4 and fhd4 (tools/ab_inproc.py; digests checked).
# Usage: tools/gpu_abq.sh <tag> <rounds> lib1.so lib2.so ...   (WL="uhd4 fhd4" by default)
set -o pipefail
TAG=$1; RND=$2; shift 2
OUT=gpurun_out/abq_$TAG
mkdir -p $OUT
for w in ${WL:-uhd4 fhd4}; do
	timeout -k 10 400 python3 -u tools/ab_inproc.py --workload $w --rounds $RND --steps 6 "$@" > $OUT/$w.json 2> $OUT/$w.err \
		|| { echo "FAIL $w"; grep -v amdgpu.ids $OUT/$w.err | tail -5; exit 1; }
	echo "== $w"; cat $OUT/$w.json
done
