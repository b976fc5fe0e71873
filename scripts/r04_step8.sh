#!/bin/bash
# Window and edge lines issued together: parity, A (joint) / B (separate passes, ab/nojoint)
# timing, and the read bytes of each side (FETCH_SIZE, one side per pass)
set -o pipefail
O=gpurun_out/r04_step8
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ip6.py tests/test_gpu_ring.py tests/test_gpu_opts.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
R=$(pwd)
run() { timeout -k 10 300 python3 -u tools/ab_lib.py ab/nojoint/librpkt_gpu.so --rounds 7 --launches 10 "$@" >> $O/ab.jsonl 2>> $O/ab.log; }
run --leg parse3 && run --leg parse5 && run --leg parse11 --flags 11 && run --leg popts5 && \
run --leg parsec3 && run --leg parse3 || exit 1
cd /tmp && export TMPDIR=/tmp
for side in A B; do
  for leg in parse3 parse5; do
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$R/$O/pmc_${side}_$leg" -o p \
        -- python3 "$R/tools/ab_lib.py" "$R/ab/nojoint/librpkt_gpu.so" --leg $leg --sides $side --rounds 1 --launches 10 \
        > "$R/$O/pmc_${side}_$leg.log" 2>&1 || exit 1
  done
done
echo done
