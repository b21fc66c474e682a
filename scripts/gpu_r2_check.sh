# GPU check: parity suite (+ the not yet collected no-alloc test), smoke, short bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r2check"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo TESTS_FAILED; tail -60 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
if [ -f tests/test_zz_no_alloc.py ]; then
timeout -k 10 300 python -u -m pytest tests/test_zz_no_alloc.py -x -v --timeout 120 --timeout-method thread > "$O/noalloc.log" 2>&1 || { echo NOALLOC_FAILED; tail -60 "$O/noalloc.log"; exit 1; }
tail -3 "$O/noalloc.log"
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > "$O/smoke.log" 2>&1 || { echo SMOKE_FAILED; tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
echo CHECK_OK
