#!/bin/bash
# pipeline on the quad chain kernel: its GPU tests, then the end-to-end device-m05 leg A/B
set -o pipefail
mkdir -p gpurun_out/q13
true
tail -3 gpurun_out/q13/tests.log
LD_LIBRARY_PATH=$PWD/webp-decoder_amd/lib timeout -k 10 600 python -u tools/e2e_ab.py --frames 1024 --reps 3 webp-decoder_amd/lib/ab/quad_drain1.so webp-decoder_amd/lib/libvp8g.so > gpurun_out/q13/e2e.json 2> gpurun_out/q13/e2e.err || { tail -20 gpurun_out/q13/e2e.err; exit 1; }
cat gpurun_out/q13/e2e.json
