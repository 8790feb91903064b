#!/bin/bash
# Round 6 call f: stamps / ablations of the current build (tools/gpu_r06_stamps.sh), the LDS
# quarter-padding A/B (bank conflicts of the loop filter's byte gathers) and its LDS PMC group.
# Libraries: bash tools/build_ab.sh qpad4 "-DVP8G_QPAD=4"; bash tools/build_ab.sh qpad16 "-DVP8G_QPAD=16".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06f 0 uhd4,synth webp-decoder_amd/lib/libvp8g.so $L/qpad4.so $L/qpad16.so || exit 1
export TMPDIR=/tmp
QUIET="--e2e-frames 0 --extra none --encode none --no-cpu-baseline"
for v in base qpad4; do
  lib=$R/webp-decoder_amd/lib/libvp8g.so; [ $v = qpad4 ] && lib=$R/$L/qpad4.so
  mkdir -p $R/gpurun_out/pmc_r06f_$v
  (cd /tmp && VP8G_LIB=$lib timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmc_r06f_$v/p -o pmc -- python3 $R/bench.py $QUIET --steps 2 --warmup 1 > $R/gpurun_out/pmc_r06f_$v/log 2>&1) || { echo "pmc $v failed"; exit 1; }
done
echo pmc_done
bash tools/gpu_r06_stamps.sh r06t || exit 1
