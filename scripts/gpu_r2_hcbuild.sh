# LZ4HC build kernel timing experiments (no parity tests: the bench leg under a kernel trace).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/r2hcb"; mkdir -p "$O"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/trace" -o t -- python3 $R/bench.py --no-cpu-baseline --no-legs --workload lz4hc --partitions 256 --steps 2 --warmup 1 > "$O/bench.json" 2> "$O/trace.err" || { echo TRACE_FAILED; tail -5 "$O/trace.err"; exit 1; }
find "$O/trace" -name "*kernel_stats.csv" -exec head -4 {} \;
rm -rf "$O/trace"
