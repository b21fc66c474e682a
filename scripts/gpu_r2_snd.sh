# snappy decode check: parity tests, then the uncompress leg.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r2snd"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_producer.py -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; tail -60 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 300 python bench.py --workload snappyd --partitions 1024 --steps 3 --warmup 1 --no-cpu-baseline > "$O/snappyd.json" 2> "$O/snappyd.err" || { echo BENCH_FAILED; tail -20 "$O/snappyd.err"; exit 1; }
python - "$O/snappyd.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["workload"], "GB/s", d["GB_per_s"], "kernel_ms", d["roofline"]["kernel_ms"])
PY
echo SND_OK
