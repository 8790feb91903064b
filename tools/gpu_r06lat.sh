#!/bin/bash
# Round 6 call lat: memory-latency counters of the quad kernel -- average VMEM / LDS instruction latency
# (the derived VmemLatency / LdsLatency), EA read / write requests and their in-flight levels (average
# latency = level / requests, per TCC), DRAM-credit and write stalls, TA stalls by TC -- for the product
# build on uhd4 and synth and for the store-ablated diag build (abl4) on uhd4.  One group per pass.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_r06lat
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
QUIET="--e2e-frames 0 --extra none --encode none --no-cpu-baseline"
run() {  # tag lib workload
  local tag=$1 lib=$2 wl=$3 i=0
  for grp in "VmemLatency LdsLatency" \
             "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum" \
             "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    VP8G_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $O/${tag}_p$i -o pmc -- python3 $R/bench.py $QUIET --workload $wl --steps 2 --warmup 1 > $O/${tag}_p$i.log 2>&1 || { echo "pass $tag $i failed rc=$?"; tail -5 $O/${tag}_p$i.log; exit 1; }
  done
}
run uhd4 $R/webp-decoder_amd/lib/libvp8g.so uhd4
run synth $R/webp-decoder_amd/lib/libvp8g.so synth
run uhd4_abl4 $R/webp-decoder_amd/lib/diag/libvp8g_abl4.so uhd4
echo lat_done
