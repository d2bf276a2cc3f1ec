#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
for e in "1 0" "0 1" "1 0" "0 1" "1 0" "0 1"; do
  set -- $e
  echo -n "EARLY_PREP=$1 EARLY_ZERO=$2: "
  MOG_EARLY_PREP=$1 MOG_EARLY_ZERO=$2 timeout -k 10 200 python -u -m pytest tests/test_gpu_x3.py -q -k fp32_step_gradients --timeout 150 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "passed|failed|assert 0" | head -3 | tr '\n' ' ' || true
  echo
done
