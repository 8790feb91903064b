#!/bin/bash
# quad experiment: per-MB diff against the shipped build on one workload (tools/quad_debug.py)
set -o pipefail
W=${1:-uhd4_yuv}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/quad_debug.py --workload $W webp-decoder_amd/lib/libvp8g.so \
	webp-decoder_amd/lib/diag/libvp8g_quad.so > gpurun_out/qdbg_$W.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/qdbg_$W.log
exit $rc
