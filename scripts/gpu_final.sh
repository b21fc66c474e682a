# Round-end evidence after the LZ4HC leg: GPU parity tests, smoke, default
# bench line (with the lz4hc leg), kernel traces of the CRC headline and of the
# LZ4HC leg.  Every GPU step has its own limit; the script stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
O="$R/gpurun_out/final"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo TESTS_FAILED; tail -40 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 200 python __graft_entry__.py > "$O/smoke.log" 2>&1 || { echo SMOKE_FAILED; tail -20 "$O/smoke.log"; exit 1; }
timeout -k 10 500 python bench.py > "$O/bench.log" 2>&1 || { echo BENCH_FAILED; tail -20 "$O/bench.log"; exit 1; }
cat "$O/bench.log"
cd /tmp && export TMPDIR=/tmp
P="$O/prof"; mkdir -p "$P"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$P/crc" -o k -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-legs > "$P/crc.log" 2>&1 || { echo TRACE1_FAILED; tail -20 "$P/crc.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$P/lz4hc" -o k -- python3 $R/bench.py --workload lz4hc --level 9 --partitions 256 --steps 3 --warmup 1 --no-cpu-baseline > "$P/lz4hc.log" 2>&1 || { echo TRACE2_FAILED; tail -20 "$P/lz4hc.log"; exit 1; }
for d in crc lz4hc; do echo "== $d"; grep -h "GB" "$P/$d.log" | cut -c1-300; head -4 "$P/$d/k_kernel_stats.csv"; done
echo ALL_OK
