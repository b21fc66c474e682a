# LZ4HC leg: HBM traffic (FETCH_SIZE / WRITE_SIZE passes, one per run) at 256 x 1 MiB, level 9.
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/hcpmc"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --workload lz4hc --level 9 --partitions 256 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -f csv -d "$O/fetch" -o k -- python3 $B > "$O/fetch.log" 2>&1 || { echo PMC1_FAILED; tail -20 "$O/fetch.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -f csv -d "$O/write" -o k -- python3 $B > "$O/write.log" 2>&1 || { echo PMC2_FAILED; tail -20 "$O/write.log"; exit 1; }
ls -R "$O" | head -20
echo ALL_OK
