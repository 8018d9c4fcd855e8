#!/bin/bash
# Micro timings on the GPU box: step sections (graph replay) and graph-timed GEMM shapes.
set -o pipefail
mkdir -p gpurun_out/micro
tools/gpu_steps.sh "300 micro/sections.log python3 tools/step_sections.py" \
  "300 micro/gemm.log python3 tools/gemm_micro.py"
