# Kernel trace of the consumer leg (CRC verify + LZ4F decompress, 1024 x 1 MiB).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/consumer"; mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/trace" -o con -- python3 $R/bench.py --workload consumer --partitions 1024 --steps 3 --warmup 1 --no-cpu-baseline > "$O/consumer.log" 2>&1 || { echo TRACE_FAILED; tail -20 "$O/consumer.log"; exit 1; }
echo OK
