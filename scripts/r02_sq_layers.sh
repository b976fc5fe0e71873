#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/sq_counters.sh layA 2 layers_kernel --tx layers9 --compact "" > gpurun_out/r02_sq_layA.json 2>gpurun_out/r02_sq_layA.err && \
COUNTERS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH" bash scripts/sq_counters.sh layB 2 layers_kernel --tx layers9 --compact "" > gpurun_out/r02_sq_layB.json 2>gpurun_out/r02_sq_layB.err && \
COUNTERS="SQ_WAVES SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM" bash scripts/sq_counters.sh layC 2 layers_kernel --tx layers9 --compact "" > gpurun_out/r02_sq_layC.json 2>gpurun_out/r02_sq_layC.err
