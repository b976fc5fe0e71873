#!/bin/bash
# time-slotted mixed streams (tools/slotbw.hip): reads and writes separated in time across
# the chip by the real-time counter, against the proportional mix, at config 2's and
# config 3's read:write ratios
set -o pipefail
O=gpurun_out/r03_slotbw
mkdir -p $O
timeout -k 10 240 ./tools/slotbw > $O/slotbw.log 2>&1
