#!/bin/bash
# PMC passes for the bench kernel (one counter group per rocprofv3 run; never combined with
# tracing domains).  Usage: bash tools/pmc_pass.sh <outdir> [bench args...]
set -u
OUT=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/$OUT/pmc$i -o pmc -- python3 $R/bench.py "$@" > $R/$OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; exit 1; }
done
echo pmc_done
