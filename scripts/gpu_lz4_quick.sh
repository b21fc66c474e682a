# LZ4 iteration loop: LZ4 parity tests, consumer + compress legs, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/l
timeout -k 10 600 python -m pytest tests/test_gpu_lz4.py -x -q > gpurun_out/l/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/l/tests.log; exit 1; }
tail -1 gpurun_out/l/tests.log
timeout -k 10 300 python bench.py --workload consumer --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/l/consumer.log 2>&1 || { echo CONSUMER_FAILED; tail gpurun_out/l/consumer.log; exit 1; }
timeout -k 10 300 python bench.py --workload lz4c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/l/lz4c.log 2>&1 || { echo LZ4C_FAILED; tail gpurun_out/l/lz4c.log; exit 1; }
cat gpurun_out/l/consumer.log gpurun_out/l/lz4c.log
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$R/gpurun_out/l/trace" -o lz4 -- python3 $R/bench.py --workload consumer --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/l/trace.log" 2>&1 || { echo TRACE_FAILED; exit 1; }
cat "$R/gpurun_out/l/trace/lz4_kernel_stats.csv"
B="$R/bench.py --workload consumer --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -T -f csv -d "$R/gpurun_out/l/pmc1" -o lz4 -- python3 $B > "$R/gpurun_out/l/pmc1.log" 2>&1 || { echo PMC1_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS -T -f csv -d "$R/gpurun_out/l/pmc2" -o lz4 -- python3 $B > "$R/gpurun_out/l/pmc2.log" 2>&1 || { echo PMC2_FAILED; tail -5 "$R/gpurun_out/l/pmc2.log"; exit 1; }
echo PMC_OK
