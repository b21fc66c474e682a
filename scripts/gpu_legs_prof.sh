# rocprofv3 kernel traces of the LZ4F legs (fast compress, consumer, producer pipeline).
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/legs"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/lz4c_fast" -o k -- python3 $R/bench.py --workload lz4c_fast --partitions 256 --steps 3 --warmup 1 --no-cpu-baseline > "$O/lz4c_fast.log" 2>&1 || { echo T1_FAILED; tail -5 "$O/lz4c_fast.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/consumer" -o k -- python3 $R/bench.py --workload consumer --partitions 1024 --steps 3 --warmup 1 --no-cpu-baseline > "$O/consumer.log" 2>&1 || { echo T2_FAILED; tail -5 "$O/consumer.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/producer" -o k -- python3 $R/bench.py --workload producer --partitions 512 --steps 2 --warmup 1 --no-cpu-baseline > "$O/producer.log" 2>&1 || { echo T3_FAILED; tail -5 "$O/producer.log"; exit 1; }
for d in lz4c_fast consumer producer; do echo "== $d"; grep workload "$O/$d.log" | cut -c1-200; head -6 "$O/$d/k_kernel_stats.csv"; done
