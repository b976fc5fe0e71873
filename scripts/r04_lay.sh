#!/bin/bash
# Layer walk, half-slot refills (RPKT_LAY_HALF): A/B timing against the in-tree build on
# the capture mix and config 2 / 5 layer legs (outputs compared byte for byte), then
# FETCH_SIZE / WRITE_SIZE of each side alone.  B sides are built on the CPU host:
#   python tools/ab_lib.py --build ab/half -DRPKT_LAY_HALF=1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04_lay
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
AB="$R/tools/ab_lib.py"
BSIDES=${BSIDES:-half}
for B in $BSIDES; do
  for leg in ${LEGS-layers9 layers2 layers5}; do
    timeout -k 10 300 python3 -u "$AB" "$R/ab/$B/librpkt_gpu.so" --leg $leg --rounds 7 --launches 20 \
        >> "$O/ab_$B.jsonl" 2>> "$O/ab_$B.log" || exit 1
  done
done
B1=${BSIDES%% *}
for side in A $BSIDES; do
  lib="$R/ab/${side}/librpkt_gpu.so"; s=B
  if [ "$side" = A ]; then lib="$R/ab/$B1/librpkt_gpu.so"; s=A; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -T --output-format csv -d "$O/pmc_${side}_$c" -o p \
        -- python3 "$AB" "$lib" --leg layers9 --sides $s --rounds 1 --launches 10 \
        > "$O/pmc_${side}_$c.log" 2>&1 || exit 1
  done
done
echo done
