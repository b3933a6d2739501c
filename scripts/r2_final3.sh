#!/bin/bash
# End-of-session validation: full GPU suite, smoke(), ResNet-50 and BERT benches,
# steady-state BERT kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
SKIP_TESTS=0 BENCHES="resnet50 bert" REHEARSE=0 PROFILE_MODEL=bert bash scripts/r2_final.sh || exit $?
