#!/bin/bash
# Throughput compressor after a change: digest of its frames against the kept baseline, then the
# compress-only and the headline (finalize) bench lines.   usage: bash scripts/gpu_r3_fast_check.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/gpu_r3_fast_digest.py > gpurun_out/fast_digest_new.txt 2>&1 || { echo DIGEST_RUN_FAILED; tail -5 gpurun_out/fast_digest_new.txt; exit 1; }
grep FAST_DIGEST gpurun_out/fast_digest_new.txt
if [ -f gpurun_out/fast_digest_base.txt ]; then
  if [ "$(grep FAST_DIGEST gpurun_out/fast_digest_base.txt)" == "$(grep FAST_DIGEST gpurun_out/fast_digest_new.txt)" ]; then echo DIGEST_SAME; else echo DIGEST_DIFFERS; fi
fi
timeout -k 10 120 python bench.py --no-cpu-baseline --no-legs --workload lz4c_fast --steps 10 --warmup 3 > gpurun_out/ab_fast.json 2>gpurun_out/ab_fast.err || { echo BENCH_FAST_FAILED; exit 1; }
timeout -k 10 120 python bench.py --no-cpu-baseline --no-legs --steps 10 --warmup 3 > gpurun_out/ab_fin.json 2>>gpurun_out/ab_fast.err || { echo BENCH_FIN_FAILED; exit 1; }
python - <<PY
import json
for f in ("gpurun_out/ab_fast.json", "gpurun_out/ab_fin.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d.get("value", d.get("GB_per_s")), d.get("compression_ratio"), d["roofline"]["kernel_ms"])
PY
