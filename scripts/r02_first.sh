set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.log
