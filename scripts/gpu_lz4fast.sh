# LZ4F throughput-mode compressor: parity tests, then the compress leg with a kernel trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/fast"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4.py -x -v --timeout 120 --timeout-method thread -k fast > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; tail -40 "$O/tests.log"; exit 1; }
tail -5 "$O/tests.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/trace" -o f -- python3 $R/bench.py --workload lz4c_fast --partitions 256 --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench.log" 2>&1 || { echo BENCH_FAILED; tail -20 "$O/bench.log"; exit 1; }
cat "$O/bench.log"; cat "$O/trace/f_kernel_stats.csv"
