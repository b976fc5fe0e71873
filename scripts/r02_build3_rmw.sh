#!/bin/bash
# build 3 read traffic with and without the write-back (partial-line read-modify-write?)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/build3_rmw
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=(--no-cpu --config 2 --also "" --tx build3 --compact "" --steps 20 --warmup 5 --no-config1)
for lib in _build _build_nowb; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -T --output-format csv -d "$OUT/$lib" -o $c \
      -- python3 "$R/tools/bench_with_lib.py" "$R/rpkt_amd/$lib/librpkt_gpu.so" "${ARGS[@]}" \
      > "$OUT/${lib}_$c.log" 2>&1 || exit 1
  done
done
echo done
