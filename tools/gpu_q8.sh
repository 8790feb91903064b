set -o pipefail
bash tools/gpu_abq.sh q8 4 webp-decoder_amd/lib/libvp8g.so webp-decoder_amd/lib/ab/quad_sc1.so && bash tools/gpu_round.sh diag r05q8
