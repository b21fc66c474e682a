# GPU parity suite, smoke and the default bench line (no profiling).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/check"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo TESTS_FAILED; tail -40 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > "$O/smoke.log" 2>&1 || { echo SMOKE_FAILED; tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 500 python bench.py > "$O/bench.log" 2>&1 || { echo BENCH_FAILED; tail -20 "$O/bench.log"; exit 1; }
grep '"metric"' "$O/bench.log" > "$O/bench_line.json"
echo CHECK_OK
