# encode-only extraction: GPU parity tests and the cfg4 throughput line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_extract.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/extract_tests.log 2>&1 || { tail -40 gpurun_out/extract_tests.log; exit 1; }
tail -3 gpurun_out/extract_tests.log
timeout -k 10 300 python tools/bench_encode.py > gpurun_out/encode.json 2> gpurun_out/encode.err || { tail -30 gpurun_out/encode.err; exit 1; }
cat gpurun_out/encode.json
