# Encoder A/B: the default library against a variant (lib/libgaphuff_$1.so), cfg4 and cfg3,
# alternating, then the encoder GPU tests on the default library.
set -o pipefail
O=gpurun_out/${2:-r05enc}; mkdir -p $O
L=$PWD/cse375-finalproj-huffman-decoding_amd/lib
for i in 1 2; do
  timeout -k 10 200 python -u scripts/bench_encode.py cfg4 cfg3 > $O/base_$i.log 2>&1 || exit 1
  echo "base $i"; cat $O/base_$i.log
  GAPHUFF_LIB=$L/libgaphuff_$1.so timeout -k 10 200 python -u scripts/bench_encode.py cfg4 cfg3 > $O/var_$i.log 2>&1 || exit 1
  echo "$1 $i"; cat $O/var_$i.log
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py -q -x -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1; tail -3 $O/tests.log
