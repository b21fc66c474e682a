# Producer/finalize tests, then the default bench line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r2bench"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_producer.py tests/test_gpu_multirank.py -x -v --timeout 600 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; tail -60 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
timeout -k 10 900 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo BENCH_FAILED; tail -30 "$O/bench.err"; exit 1; }
python - "$O/bench.json" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
legs = d.pop("legs", {})
print(json.dumps(d, indent=1))
for k, v in legs.items():
    print(k, json.dumps(v)[:600])
PY
echo BENCH_OK
