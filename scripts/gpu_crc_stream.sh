# CRC32C streamed kernel: parity tests, then headline bench streamed vs per-batch.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/crcs"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc.py -x -v --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error" "$O/tests.log" | head; tail -20 "$O/tests.log"; exit 1; }
grep -c PASSED "$O/tests.log"
timeout -k 10 200 python bench.py --no-legs --no-cpu-baseline > "$O/stream.log" 2>&1 || { echo BENCH1_FAILED; tail "$O/stream.log"; exit 1; }
RDK_HIP_CRC_NOSTREAM=1 timeout -k 10 200 python bench.py --no-legs --no-cpu-baseline > "$O/nostream.log" 2>&1 || { echo BENCH2_FAILED; tail "$O/nostream.log"; exit 1; }
python - <<'P'
import json
for f in ("stream", "nostream"):
    d = json.loads(open(f"gpurun_out/crcs/{f}.log").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["roofline"]["frac"])
P
