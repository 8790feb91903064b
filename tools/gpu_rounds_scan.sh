#!/bin/bash
# Per-frame kernel time of the shipped build against the batch size (uhd4 frames per launch): how much
# the chain's fill / drain and its last partial round of pairs cost.
set -o pipefail
mkdir -p gpurun_out/rounds_scan
for n in 256 384 512 640 768 1024; do
	timeout -k 10 240 python3 -u tools/ab_inproc.py --workload uhd4 --frames $n --rounds 3 --steps 6 \
		webp-decoder_amd/lib/libvp8g.so > gpurun_out/rounds_scan/n$n.json || exit 1
	echo "n=$n $(cat gpurun_out/rounds_scan/n$n.json)"
done
