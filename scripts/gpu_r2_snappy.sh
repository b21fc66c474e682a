# snappy check: parity tests (compress first, so that a decoder problem cannot hide it).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r2snappy"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py -x -v --timeout 120 --timeout-method thread -k "compress" > "$O/tests_c.log" 2>&1 || { echo COMPRESS_TESTS_FAILED; tail -40 "$O/tests_c.log"; exit 1; }
tail -3 "$O/tests_c.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py -x -v --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; tail -60 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
