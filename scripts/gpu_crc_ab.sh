# CRC v1/v3 A/B: CRC parity tests, v1 bench, default bench (v3 + LZ4F legs +
# CPU baselines), then rocprofv3 kernel-trace stats + counter passes for v3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_crc.py -x -q > gpurun_out/gpu_tests_crc.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests_crc.log; exit 1; }
tail -1 gpurun_out/gpu_tests_crc.log
RDK_HIP_CRC_V1=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-legs > gpurun_out/bench_v1.log 2>&1 || { echo BENCH1_FAILED; tail gpurun_out/bench_v1.log; exit 1; }
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_v3.log 2>&1 || { echo BENCH3_FAILED; tail -20 gpurun_out/bench_v3.log; exit 1; }
cat gpurun_out/bench_v1.log gpurun_out/bench_v3.log
bash scripts/profile_crc.sh
