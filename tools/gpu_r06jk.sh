#!/bin/bash
# Round 6 calls j and k in one box: memory-policy A/B, then the priority sweep and store-ablation stamps.
set -u
bash tools/gpu_r06j.sh && bash tools/gpu_r06k.sh
