set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 200 python -u scripts/quick_one.py cfg4:1000000000:0.1 20 > gpurun_out/r03a/q.log 2>&1 &&
timeout -k 10 200 python -u scripts/quick_one.py cfg3:1000000000:0.9 20 >> gpurun_out/r03a/q.log 2>&1 &&
timeout -k 10 200 python -u scripts/quick_one.py cfg5:1000000000:0.5 20 >> gpurun_out/r03a/q.log 2>&1
cat gpurun_out/r03a/q.log
