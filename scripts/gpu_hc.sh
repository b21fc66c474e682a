# LZ4HC work-queue check: parity tests for the HC engine, then the lz4hc leg at
# 64 and 256 frames (levels 9 and 3), kernel trace of the 256-frame level-9 run.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
O="$R/gpurun_out/hc"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4hc.py -m gpu -x -v --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for p in 64 256; do for l in 9 3; do
timeout -k 10 200 python bench.py --workload lz4hc --level $l --partitions $p --steps 3 --warmup 1 --no-cpu-baseline > "$O/b_${p}_${l}.log" 2>&1 || { echo BENCH_FAILED; tail -20 "$O/b_${p}_${l}.log"; exit 1; }
echo "p=$p l=$l $(tail -1 $O/b_${p}_${l}.log)"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/prof" -o k -- python3 $R/bench.py --workload lz4hc --level 9 --partitions 256 --steps 3 --warmup 1 --no-cpu-baseline > "$O/prof.log" 2>&1 || { echo TRACE_FAILED; tail -20 "$O/prof.log"; exit 1; }
head -4 "$O/prof/k_kernel_stats.csv"
echo ALL_OK
