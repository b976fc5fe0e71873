#!/bin/bash
# GPU test run in stages on the box: each stage under its own time limit, logs under
# gpurun_out/; a stage whose tests fail (pytest rc 1) lets the next one run, anything else
# (a hang, an abort, a time limit) ends the script there.
#   bash scripts/gpu_tests.sh <tag> "<pytest selection>" ["<pytest selection>" ...]
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
k=0
for sel in "$@"; do
    k=$((k + 1))
    timeout -k 10 600 python -u -m pytest $sel -x -q --timeout 240 --timeout-method thread \
        > gpurun_out/pytest_${TAG}_$k.log 2>&1
    rc=$?
    echo "stage $k ($sel): rc=$rc"; tail -3 gpurun_out/pytest_${TAG}_$k.log
    if [ $rc -gt 1 ]; then exit $rc; fi
done
