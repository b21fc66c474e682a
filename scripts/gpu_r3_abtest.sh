#!/bin/bash
# the LZ4 compress tests against one A/B build, then the A/B timing
set -o pipefail
RDK_HIP_LIB="$GRAFT_REPO_ROOT/abtmp/$1" timeout -k 10 600 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread -k "fast or finalize or perf_tool" 2>&1 | tail -3 || exit 1
bash scripts/gpu_r3_ab.sh "base $2 base $2" --workload lz4c_fast --partitions 512 --steps 10
