#!/bin/bash
# one library under several environment settings (env switches are read once per process, so each
# setting is its own ab_inproc process on the same box): kernel medians per workload
# Usage: tools/gpu_envab.sh [workloads, default "uhd4 fhd4"]
set -o pipefail
mkdir -p gpurun_out/envab
for w in ${1:-uhd4 fhd4}; do
	for cfg in "X=0" "VP8G_SPLITCHAIN=0" "VP8G_SPLITCHAIN=0 VP8G_CHAIN_IL=1" "VP8G_CHAIN_IL=0" "VP8G_SPLITCHAIN=1" "X=1"; do
		env $cfg timeout -k 10 300 python3 -u tools/ab_inproc.py --workload $w --rounds 3 --steps 6 webp-decoder_amd/lib/libvp8g.so \
			> gpurun_out/envab/out.json 2> gpurun_out/envab/err.txt || { tail -5 gpurun_out/envab/err.txt; exit 1; }
		echo "$w $cfg $(cat gpurun_out/envab/out.json)"
	done
done
