#!/bin/bash
# build kernel: edge lines with the window (product) vs a pass after it (B); traffic + time
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/build_ew
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread \
    > "$OUT/tx_tests.log" 2>&1 || exit 1
for leg in build3 build2; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_ew0/librpkt_gpu.so --leg $leg --rounds 8 --launches 20 \
    > "$OUT/ab_$leg.log" 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
ARGS=(--no-cpu --config 2 --also "" --tx build3 --compact "" --steps 20 --warmup 5 --no-config1)
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -T --output-format csv -d "$OUT/pmc" -o $c \
    -- python3 "$R/bench.py" "${ARGS[@]}" > "$OUT/pmc_$c.log" 2>&1 || exit 1
done
echo done
