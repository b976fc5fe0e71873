#!/bin/bash
# SQ counters of the layer walk and the field getters on the final build
set -o pipefail
bash scripts/sq_counters.sh final_layers 2 layers_kernel --tx layers9 > gpurun_out/sq_final_layers.json 2> gpurun_out/sq_final_layers.err && \
bash scripts/sq_counters.sh final_fields 2 fields_kernel --tx fields9 > gpurun_out/sq_final_fields.json 2> gpurun_out/sq_final_fields.err
