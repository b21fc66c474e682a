set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
nproc > gpurun_out/nproc.txt; cat /proc/cpuinfo | grep "model name" | head -1 >> gpurun_out/nproc.txt
timeout -k 10 400 python -m pytest tests/test_gpu_crc.py -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 200 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; exit 1; }
cat gpurun_out/bench.log
