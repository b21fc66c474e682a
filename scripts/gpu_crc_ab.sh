# CRC v1/v2 A/B + full bench with LZ4 legs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_crc.py -x -q > gpurun_out/gpu_tests_crc.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests_crc.log; exit 1; }
tail -1 gpurun_out/gpu_tests_crc.log
RDK_HIP_CRC_V1=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-legs > gpurun_out/bench_v1.log 2>&1 || { echo BENCH1_FAILED; tail gpurun_out/bench_v1.log; exit 1; }
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_v2.log 2>&1 || { echo BENCH2_FAILED; tail -20 gpurun_out/bench_v2.log; exit 1; }
cat gpurun_out/bench_v1.log gpurun_out/bench_v2.log
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -T -f csv -d "$R/gpurun_out/prof_v2/pmc_sq" -o crc -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > "$R/gpurun_out/prof_v2_sq.log" 2>&1 || { echo PMC_FAILED; exit 1; }
