# A/B check after a change that touches every LZ4 kernel: parity tests, then the main legs.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r2ab"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_lz4hc.py tests/test_gpu_producer.py tests/test_gpu_snappy.py tests/test_zz_no_alloc.py -x -q --timeout 600 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for W in "finalize --partitions 512" "lz4c_fast --partitions 256" "lz4hc --partitions 256" "consumer --partitions 1024" "snappyc --partitions 256" "snappyd --partitions 1024"; do
timeout -k 10 300 python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-legs 2> "$O/err.log" | grep -o "\"workload\": \"[a-z_0-9]*\"\|\"value\": [0-9.]*\|\"GB_per_s\": [0-9.]*" | tr '\n' ' ' || { echo BENCH_FAILED "$W"; tail -20 "$O/err.log"; exit 1; }
echo " <- $W"
done
