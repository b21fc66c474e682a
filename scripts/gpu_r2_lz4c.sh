# Exact LZ4F compressor: parity tests, then the lz4c bench leg (windowed and sequential engines).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r2lz4c"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_producer.py tests/test_zz_no_alloc.py -x -v --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; tail -60 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
timeout -k 10 300 python bench.py --workload lz4c --partitions 256 --steps 5 --warmup 2 --no-cpu-baseline > "$O/lz4c_window.json" 2> "$O/lz4c_window.err" || { echo BENCH_FAILED; tail -20 "$O/lz4c_window.err"; exit 1; }
cat "$O/lz4c_window.json"
RDK_HIP_LZ4_EXACT_SEQ=1 timeout -k 10 300 python bench.py --workload lz4c --partitions 256 --steps 5 --warmup 2 --no-cpu-baseline > "$O/lz4c_seq.json" 2> "$O/lz4c_seq.err" || { echo BENCH_FAILED; tail -20 "$O/lz4c_seq.err"; exit 1; }
cat "$O/lz4c_seq.json"
timeout -k 10 300 python bench.py --workload lz4c_fast --partitions 256 --steps 5 --warmup 2 --no-cpu-baseline > "$O/lz4c_fast.json" 2> "$O/lz4c_fast.err" || { echo BENCH_FAILED; tail -20 "$O/lz4c_fast.err"; exit 1; }
cat "$O/lz4c_fast.json"
echo LZ4C_OK
