# LZ4HC check: parity tests, then the level 9 / 10 / 12 legs (kernel times only).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r2hc"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lz4hc.py -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; tail -60 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for lv in 9 10 12; do
  timeout -k 10 300 python bench.py --workload lz4hc --level $lv --partitions 256 --steps 2 --warmup 1 --no-cpu-baseline > "$O/l$lv.json" 2> "$O/l$lv.err" || { echo BENCH_FAILED $lv; tail -20 "$O/l$lv.err"; exit 1; }
  python - "$O/l$lv.json" $lv <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("level", sys.argv[2], "GB/s", d["GB_per_s"], "kernel_ms", d["roofline"]["kernel_ms"], "ratio", d.get("compression_ratio"))
PY
done
echo HC_OK
