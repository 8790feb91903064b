#!/bin/bash
# quad kernel templated on whole pieces (lean instantiation for whole-piece batches, byte path otherwise):
# then the A/B against the whole-piece-only build
set -o pipefail
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_quad.py tests/test_gpu_batch.py tests/test_gpu_parity.py > gpurun_out/q19_tests.log 2>&1 || { grep -E "PASS|FAIL|Error" gpurun_out/q19_tests.log | tail -20; tail -30 gpurun_out/q19_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/q19_tests.log | tail -2
bash tools/gpu_abq.sh q19 4 webp-decoder_amd/lib/ab/quad_c2.so webp-decoder_amd/lib/libvp8g.so
