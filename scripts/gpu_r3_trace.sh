#!/bin/bash
# kernel-trace stats of one bench workload: per-kernel average duration
#   usage: bash scripts/gpu_r3_trace.sh TAG bench.py-arguments...
set -o pipefail
TAG="$1"; shift
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/trace_$TAG"; rm -rf "$O"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/t" -o t -- python3 $R/bench.py --no-cpu-baseline --no-legs --steps 5 --warmup 1 "$@" > "$O/bench.json" 2> "$O/err" || { tail -5 "$O/err"; exit 1; }
find "$O/t" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
rm -rf "$O/t"
echo "== $TAG"; head -8 "$O/kernel_stats.csv" | cut -c1-160
