#!/bin/bash
# the whole GPU test suite, as the round driver runs it (one process), log -> gpurun_out/suite/pytest.log
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/suite
timeout -k 10 1150 python -u -m pytest tests -m gpu -v -rf --timeout 1000 --timeout-method thread -p no:cacheprovider > gpurun_out/suite/pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" gpurun_out/suite/pytest.log | tail -15
exit $rc
