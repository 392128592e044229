# Self-sync timing with the default (stream-derived) halo, then the sync GPU tests.
set -o pipefail
O=gpurun_out/${1:-r05s3}; mkdir -p $O
GH_SYNC_VERBOSE=1 timeout -k 10 200 python -u scripts/bench_sync.py cfg2 cfg3 cfg4 > $O/def.log 2>&1 || exit 1
grep -v "^gh_sync" $O/def.log; grep "^gh_sync" $O/def.log | sort | uniq -c
timeout -k 10 300 python -u -m pytest tests/test_sync.py -q -x -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1; tail -3 $O/tests.log
