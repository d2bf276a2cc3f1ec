#!/bin/bash
# the captured-step / stale-memory suite with the side streams shared by every model
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 MOG_SHARED_STREAMS=1
for k in "stale" "stale" "graph_replay" "not stale"; do
  echo -n "-k $k: "
  timeout -k 10 200 python -u -m pytest tests/test_gpu_graph.py -q -k "$k" --timeout 150 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "passed|failed|^FAILED" | cut -c1-200 | tr '\n' ' ' || true
  echo
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_graph.py -q --timeout 150 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "passed|failed|^FAILED" | cut -c1-200 || true
