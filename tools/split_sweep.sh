#!/bin/bash
# Drop-in call latency over waves-per-workgroup x workgroups-per-frame (split mode).
for w in 8 16; do
  for k in 1 2 3 4 5 6 8; do
    echo "waves=$w split=$k $(VP8G_WAVES=$w VP8G_SPLIT=$k timeout -k 10 120 python tools/dropin_latency.py 5)" || exit 1
  done
done
