#!/bin/bash
# Round 6 call g: GPU tests on the tile-shift build, A/B against the previous build (wy) and the
# quarter-padding variant, LDS PMC of the tile-shift build.
# Libraries: bash tools/build_ab.sh wy ""; bash tools/build_ab.sh tsh4 "-DVP8G_TSHIFT=4"; qpad4 as in gpu_r06f.sh.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06g 1 uhd4,synth,fhd4 $L/wy.so $L/tsh4.so $L/qpad4.so || exit 1
export TMPDIR=/tmp
QUIET="--e2e-frames 0 --extra none --encode none --no-cpu-baseline"
for wl in uhd4 synth; do
  mkdir -p $R/gpurun_out/pmc_r06g_$wl
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmc_r06g_$wl/p -o pmc -- python3 $R/bench.py $QUIET --workload $wl --steps 2 --warmup 1 > $R/gpurun_out/pmc_r06g_$wl/log 2>&1) || { echo "pmc $wl failed"; exit 1; }
done
echo pmc_done
