#!/bin/bash
# Round 6 call ic: instruction-cache and instruction-fetch counters of the quad kernel (uhd4 and synth):
# lists the counters rocprofv3 offers on this part first and runs a pass only with those found.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_r06ic
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > $O/list.txt 2>&1 || { echo "list failed rc=$?"; exit 1; }
want=""
for c in SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES; do
  grep -q "\b$c\b" $O/list.txt && want="$want $c"
done
echo "counters:$want"
[ -n "$want" ] || { echo "none found"; exit 0; }
QUIET="--e2e-frames 0 --extra none --encode none --no-cpu-baseline"
for wl in uhd4 synth; do
  timeout -k 10 300 rocprofv3 --pmc $want --output-format csv -d $O/$wl -o pmc -- python3 $R/bench.py $QUIET --workload $wl --steps 2 --warmup 1 > $O/$wl.log 2>&1 || { echo "pmc $wl failed rc=$?"; tail -5 $O/$wl.log; exit 1; }
done
echo ic_done
