# CRC v4 (16-lane groups, byte tables) bring-up: CRC parity tests, then the
# headline bench for v4 and v3 back to back, then a v4 kernel trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
O="$R/gpurun_out/crc4"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc.py -x -v --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { echo TESTS_FAILED; tail -40 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
timeout -k 10 200 python bench.py --no-cpu-baseline --no-legs > "$O/bench_v4.log" 2>&1 || { echo BENCH4_FAILED; tail -20 "$O/bench_v4.log"; exit 1; }
RDK_HIP_CRC_V=3 timeout -k 10 200 python bench.py --no-cpu-baseline --no-legs > "$O/bench_v3.log" 2>&1 || { echo BENCH3_FAILED; tail -20 "$O/bench_v3.log"; exit 1; }
grep -h '"metric"' "$O/bench_v4.log" "$O/bench_v3.log" | python3 -c "import sys,json; [print(json.loads(l)['value'], json.loads(l)['roofline']) for l in sys.stdin]"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/trace" -o crc -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-legs > "$O/trace.log" 2>&1 || { echo TRACE_FAILED; tail -20 "$O/trace.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -T -f csv -d "$O/pmc_sq" -o crc -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-legs > "$O/pmc_sq.log" 2>&1 || { echo PMC_FAILED; tail -20 "$O/pmc_sq.log"; exit 1; }
echo ALL_OK
