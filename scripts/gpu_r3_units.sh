# unit engine: model equality + the fast-compress tests, then timing (default build, the
# u16-table variant, the phase-profile build) and the one-wave-per-block engine
set -o pipefail
cd "$GRAFT_REPO_ROOT"
echo "== tests (default build)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4.py -x -q -k "fast" --timeout 120 --timeout-method thread 2>&1 | tail -15 || exit 1
echo "== bench units"
timeout -k 10 200 python bench.py --workload lz4c_fast --partitions 256 --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | tail -1 || exit 1
if [ -f abtmp/librdkafka_hip_u16.so ]; then
echo "== tests (u16 table)"
RDK_HIP_LIB=$PWD/abtmp/librdkafka_hip_u16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4.py -q -k "fast" --timeout 120 --timeout-method thread 2>&1 | tail -8
echo "== bench units u16"
RDK_HIP_LIB=$PWD/abtmp/librdkafka_hip_u16.so timeout -k 10 200 python bench.py --workload lz4c_fast --partitions 256 --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | tail -1
fi
if [ -f abtmp/librdkafka_hip_prof.so ]; then
echo "== phase profile"
RDK_HIP_LIB=$PWD/abtmp/librdkafka_hip_prof.so timeout -k 10 200 python scripts/gpu_r3_prof.py 2>&1 | tail -3
fi
echo "== bench finalize_fast"
timeout -k 10 200 python bench.py --workload finalize_fast --partitions 512 --steps 10 --warmup 2 --no-cpu-baseline --no-legs 2>&1 | tail -1 || exit 1
