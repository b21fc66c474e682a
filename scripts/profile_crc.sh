# rocprofv3 evidence for the CRC32C headline: kernel-trace stats, then one
# counter pass per group (FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/prof"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$R/gpurun_out/prof/trace" -o crc -- python3 $B > "$R/gpurun_out/prof/trace.log" 2>&1 || { echo TRACE_FAILED; tail -20 "$R/gpurun_out/prof/trace.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d "$R/gpurun_out/prof/pmc_fetch" -o crc -- python3 $B > "$R/gpurun_out/prof/pmc_fetch.log" 2>&1 || { echo PMC1_FAILED; tail -20 "$R/gpurun_out/prof/pmc_fetch.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d "$R/gpurun_out/prof/pmc_write" -o crc -- python3 $B > "$R/gpurun_out/prof/pmc_write.log" 2>&1 || { echo PMC2_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -T -f csv -d "$R/gpurun_out/prof/pmc_sq" -o crc -- python3 $B > "$R/gpurun_out/prof/pmc_sq.log" 2>&1 || { echo PMC3_FAILED; tail -20 "$R/gpurun_out/prof/pmc_sq.log"; exit 1; }
find "$R/gpurun_out/prof" -name "*.csv" | head -20
