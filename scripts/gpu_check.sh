#!/bin/bash
# One GPU-box session: the GEMM/conv kernel checks + tile microbench
# (scripts/gpu_gemm_ab.sh), then the driver-form suite (scripts/gpu_driver_suite.sh).
# Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
EXTRA_TESTS="${EXTRA_TESTS:-tests/test_gemm_f32_gpu.py}" bash scripts/gpu_gemm_ab.sh || exit $?
[ "${SUITE:-1}" = "1" ] || exit 0
bash scripts/gpu_driver_suite.sh
