set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/prod"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_producer.py -x -v --timeout 200 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" "$O/tests.log" | head -20; tail -30 "$O/tests.log"; exit 1; }
grep -E "PASSED|passed" "$O/tests.log" | tail -3
