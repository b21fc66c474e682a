# CRC iteration loop: parity tests, headline bench, kernel trace + SQ counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/q
timeout -k 10 400 python -m pytest tests/test_gpu_crc.py -x -q > gpurun_out/q/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/q/tests.log; exit 1; }
tail -1 gpurun_out/q/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-legs > gpurun_out/q/bench.log 2>&1 || { echo BENCH_FAILED; tail gpurun_out/q/bench.log; exit 1; }
cat gpurun_out/q/bench.log
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
B="$R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-legs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$R/gpurun_out/q/trace" -o crc -- python3 $B > "$R/gpurun_out/q/trace.log" 2>&1 || { echo TRACE_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -T -f csv -d "$R/gpurun_out/q/pmc_sq" -o crc -- python3 $B > "$R/gpurun_out/q/pmc_sq.log" 2>&1 || { echo PMC_FAILED; exit 1; }
cat "$R/gpurun_out/q/trace/crc_kernel_stats.csv"
