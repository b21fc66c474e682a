# Kernel traces of the record writer, record index and MsgVersion 0/1 CRC legs (bench.py workloads).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/records"; mkdir -p "$O"
for w in ${WORKLOADS:-serialize index legacy}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/$w" -o rec -- python3 $R/bench.py --workload $w --partitions 256 --steps 5 --warmup 1 --no-cpu-baseline > "$O/$w.log" 2>&1 || { echo "${w}_TRACE_FAILED"; tail -20 "$O/$w.log"; exit 1; }
done
echo OK
