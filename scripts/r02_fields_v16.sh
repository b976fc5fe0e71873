#!/bin/bash
# fields: 16-B value stores (product) vs 8-B (B); parity, time, write traffic
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/fields_v16
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fields.py -x -q --timeout 120 --timeout-method thread \
    > "$OUT/tests.log" 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_v8/librpkt_gpu.so --leg fields9 --rounds 8 --launches 20 \
    > "$OUT/ab_fields9.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
ARGS=(--no-cpu --config 2 --also "" --tx fields9 --compact "" --steps 20 --warmup 5 --no-config1)
for lib in _build _build_v8; do
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/$lib" -o write \
    -- python3 "$R/tools/bench_with_lib.py" "$R/rpkt_amd/$lib/librpkt_gpu.so" "${ARGS[@]}" \
    > "$OUT/${lib}_write.log" 2>&1 || exit 1
done
echo done
