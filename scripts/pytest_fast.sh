#!/bin/bash
# GPU tests of the given files without the slow (1 GB) cases, for lease steps whose
# arguments cannot carry a quoted marker expression: bash scripts/pytest_fast.sh FILE...
exec python -u -m pytest "$@" -m "gpu and not slow" -x -q -rf --timeout 120 --timeout-method thread
