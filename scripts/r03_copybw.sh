#!/bin/bash
# HBM copy ceiling by access shape (tools/copybw.hip)
set -o pipefail
mkdir -p gpurun_out/r03_copybw
timeout -k 10 180 ./tools/copybw > gpurun_out/r03_copybw/copybw.log 2>&1
