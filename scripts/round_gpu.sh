#!/bin/bash
# Round GPU evidence on one MI355X (R=r04 bash scripts/round_gpu.sh [part]), through
# the parameterised lease runner (scripts/lease.sh):
#   part a: GPU tests (fast and slow), smoke(), the default bench line (cfg4 + the cfg5
#           sub-record, CPU baselines), the one-rank RCCL rehearsal (--force-dist),
#           cfg3 / cfg2 bench lines;
#   part b: rocprofv3 kernel stats per workload, FETCH_SIZE / WRITE_SIZE passes
#           (-> pmc_traffic.json), SQ passes of the cfg4 tile kernel;
#   part c: GPU encoder, self-sync, long codes, shard concurrency (bc: b then c).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
R=${R:-r04}
O=gpurun_out/$R
case ${1:-a} in
  a)
    bash scripts/lease.sh "$O" tests slow smoke "bench cfg4" \
      "cmd dist1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --force-dist --out-json $O/dist1.json" \
      "bench cfg3 --workload cfg3 --sub none --cpu-sample 0" "bench cfg2 --workload cfg2 --sub none --cpu-sample 0" ;;
  b)
    bash scripts/lease.sh "$O" "stats cfg4 cfg4" "stats cfg3 cfg3" "stats cfg5 cfg5" "stats cfg2 cfg2" \
      "traffic cfg4 cfg4" "traffic cfg3 cfg3" "traffic cfg5 cfg5" "traffic cfg2 cfg2" "sq cfg4 cfg4" "sq cfg3 cfg3" ;;
  c)
    bash scripts/lease.sh "$O" "cmd encode 300 python -u scripts/bench_encode.py" \
      "cmd sync 300 python -u scripts/bench_sync.py" "cmd longcodes 500 python -u scripts/time_longcodes.py --q 0.5,0.6,0.7" \
      "cmd shards 300 python -u scripts/bench_shards.py" ;;
  bc)
    bash scripts/round_gpu.sh b && bash scripts/round_gpu.sh c ;;
esac
