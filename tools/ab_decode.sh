#!/bin/bash
# A/B the decode-path variants (phase timers), one process each.
for fuse in 2 3; do for sl in 64 32; do
  echo "fuse=$fuse slices=$sl"; GENIE_DECODE_FUSE=$fuse GENIE_FFN_SLICES=$sl timeout -k 10 120 python tools/time_phases.py 2>&1 | grep -E "t2s only" | tail -1
done; done
