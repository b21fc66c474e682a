# Encoder check: parity tests of the compressors, then their bench legs (kernel times only).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r2enc"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_lz4hc.py tests/test_gpu_snappy.py tests/test_gpu_producer.py -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; tail -60 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for w in ${LEGS:-lz4c snappyc lz4c_fast lz4hc}; do
  timeout -k 10 300 python bench.py --workload $w --partitions 256 --steps 5 --warmup 2 --no-cpu-baseline > "$O/$w.json" 2> "$O/$w.err" || { echo BENCH_FAILED $w; tail -20 "$O/$w.err"; exit 1; }
  python - "$O/$w.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["workload"], "GB/s", d["GB_per_s"], "kernel_ms", d["roofline"]["kernel_ms"], "ratio", d.get("compression_ratio"))
PY
done
echo ENC_OK
