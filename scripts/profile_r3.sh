# rocprofv3 evidence for one bench leg: kernel-trace stats, then FETCH_SIZE, WRITE_SIZE and
# the SQ instruction counters in passes of their own, summarised into
# gpurun_out/prof_r3/summaries/<leg>.json (copy to profiles/r03/).
#   usage: bash scripts/profile_r3.sh LEG "KERNEL_SUBSTR[,KERNEL_SUBSTR...]" bench.py-arguments...
set -o pipefail
LEG="$1"; KERNELS="$2"; shift 2
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/prof_r3/$LEG"; rm -rf "$O"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-legs $*"
echo "profile $LEG: trace"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/trace" -o t -- python3 $B > "$O/bench.json" 2> "$O/trace.err" || { echo "TRACE_FAILED $LEG"; tail -5 "$O/trace.err"; exit 1; }
echo "profile $LEG: FETCH_SIZE"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -T -f csv -d "$O/pmc_fetch" -o t -- python3 $B > "$O/fetch.log" 2>&1 || { echo "FETCH_FAILED $LEG"; tail -5 "$O/fetch.log"; exit 1; }
echo "profile $LEG: WRITE_SIZE"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -T -f csv -d "$O/pmc_write" -o t -- python3 $B > "$O/write.log" 2>&1 || { echo "WRITE_FAILED $LEG"; tail -5 "$O/write.log"; exit 1; }
echo "profile $LEG: SQ instruction counters"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY -T -f csv -d "$O/pmc_sq" -o t -- python3 $B > "$O/sq.log" 2>&1 || { echo "SQ_FAILED $LEG"; tail -5 "$O/sq.log"; exit 1; }
mkdir -p "$R/gpurun_out/prof_r3/summaries"
python3 "$R/scripts/profile_summary.py" "$O" "$LEG" "$KERNELS" "$R/gpurun_out/prof_r3/summaries/$LEG.json" || exit 1
find "$O/trace" -name "*kernel_stats.csv" -exec cp {} "$R/gpurun_out/prof_r3/summaries/${LEG}_kernel_stats.csv" \;
# the raw per-dispatch files are large: keep the summaries only
rm -rf "$O/trace" "$O/pmc_fetch" "$O/pmc_write" "$O/pmc_sq"
