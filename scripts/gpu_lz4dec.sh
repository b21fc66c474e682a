# LZ4F decoder iteration: full LZ4 GPU parity suite, then the consumer leg with a kernel trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/dec"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_lz4.py -x -v --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" "$O/tests.log" | head -20; tail -30 "$O/tests.log"; exit 1; }
grep -c PASSED "$O/tests.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/trace" -o d -- python3 $R/bench.py --workload consumer --partitions 256 --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench.log" 2>&1 || { echo BENCH_FAILED; tail -20 "$O/bench.log"; exit 1; }
grep workload "$O/bench.log"; cat "$O/trace/d_kernel_stats.csv" | head -8
