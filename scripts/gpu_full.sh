# Full round evidence in one box session: GPU parity tests, smoke, default
# bench line, then rocprofv3 kernel trace + PMC passes for the CRC headline
# and a kernel trace of the LZ4F legs.  Every GPU step has its own limit.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
mkdir -p gpurun_out/full
O="$R/gpurun_out/full"
nproc > "$O/host.txt"; grep -m1 "model name" /proc/cpuinfo >> "$O/host.txt"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo TESTS_FAILED; tail -40 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 200 python __graft_entry__.py > "$O/smoke.log" 2>&1 || { echo SMOKE_FAILED; tail -20 "$O/smoke.log"; exit 1; }
timeout -k 10 400 python bench.py > "$O/bench.log" 2>&1 || { echo BENCH_FAILED; tail -20 "$O/bench.log"; exit 1; }
cat "$O/bench.log"
cd /tmp && export TMPDIR=/tmp
P="$O/prof"; mkdir -p "$P"
B="$R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-legs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$P/trace" -o crc -- python3 $B > "$P/trace.log" 2>&1 || { echo TRACE_FAILED; tail -20 "$P/trace.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -f csv -d "$P/pmc_fetch" -o crc -- python3 $B > "$P/pmc_fetch.log" 2>&1 || { echo PMC1_FAILED; tail -20 "$P/pmc_fetch.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -f csv -d "$P/pmc_write" -o crc -- python3 $B > "$P/pmc_write.log" 2>&1 || { echo PMC2_FAILED; tail -20 "$P/pmc_write.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -T -f csv -d "$P/pmc_sq" -o crc -- python3 $B > "$P/pmc_sq.log" 2>&1 || { echo PMC3_FAILED; tail -20 "$P/pmc_sq.log"; exit 1; }
L="$O/lz4"; mkdir -p "$L"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$L/consumer" -o lz4 -- python3 $R/bench.py --workload consumer --partitions 256 --steps 3 --warmup 1 --no-cpu-baseline > "$L/consumer.log" 2>&1 || { echo LZ4D_TRACE_FAILED; tail -20 "$L/consumer.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$L/lz4c" -o lz4 -- python3 $R/bench.py --workload lz4c --partitions 256 --steps 3 --warmup 1 --no-cpu-baseline > "$L/lz4c.log" 2>&1 || { echo LZ4C_TRACE_FAILED; tail -20 "$L/lz4c.log"; exit 1; }
echo ALL_OK
