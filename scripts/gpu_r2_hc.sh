# LZ4HC check: parity tests, then the level-9 and level-12 legs.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r2hc"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_lz4hc.py tests/test_gpu_lz4.py -x -v --timeout 600 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; tail -60 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
for L in 9 10 12; do
timeout -k 10 600 python bench.py --workload lz4hc --level $L --partitions 64 --steps 2 --warmup 1 --no-cpu-baseline > "$O/hc$L.json" 2> "$O/hc$L.err" || { echo BENCH_FAILED $L; tail -30 "$O/hc$L.err"; exit 1; }
cat "$O/hc$L.json"
done
