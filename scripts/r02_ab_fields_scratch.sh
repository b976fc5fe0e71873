#!/bin/bash
# field getters without scratch (A: offset picked by a mux tree, load9_bytes by value)
# vs the previous build (B: the compiler's indexed scratch copy of the layer record),
# then the walk-leg profile (trace + FETCH/WRITE) of the new build
set -o pipefail
OUT=gpurun_out/ab_fields_scratch
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fields.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_base/librpkt_gpu.so --leg fields9 --rounds 8 --launches 20 \
    > $OUT/ab_fields9.log 2>&1 || exit 1
bash scripts/profile.sh walks 2 --tx layers9,opts5,forward2,build2,fields9 > $OUT/profile.log 2>&1
