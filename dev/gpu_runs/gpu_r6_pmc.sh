#!/bin/bash
# round-6 PMC: encoder kernels' MFMA busy / LDS conflicts (scripts/gpu_pmc_encoder.sh)
set -o pipefail
OUT=gpurun_out/r6pmc bash scripts/gpu_pmc_encoder.sh
