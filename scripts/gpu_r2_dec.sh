# Decoder check: the LZ4 parity tests, then the consumer leg.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r2dec"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_lz4hc.py tests/test_zz_no_alloc.py tests/test_gpu_errors.py -x -v --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; tail -60 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
timeout -k 10 300 python bench.py --workload consumer --partitions 1024 --steps 3 --warmup 1 --no-cpu-baseline > "$O/consumer.json" 2> "$O/consumer.err" || { echo BENCH_FAILED; tail -30 "$O/consumer.err"; exit 1; }
cat "$O/consumer.json"
