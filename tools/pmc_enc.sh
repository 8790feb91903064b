#!/bin/bash
# PMC passes over the bench (with the m08/m09 encode stage); one counter group per rocprofv3 run.
# Usage: bash tools/pmc_enc.sh <outdir> <encode format>
set -u
OUT=$1; FMT=$2
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_FLAT_WRITE_WAVEFRONTS_sum" "TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/$OUT/pmc$i -o pmc -- python3 $R/bench.py --no-cpu-baseline --e2e-frames 0 --steps 2 --warmup 1 --frames 128 --encode $FMT > $R/$OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; exit 1; }
done
echo pmc_done
