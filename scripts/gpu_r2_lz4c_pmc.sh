# Instruction mix / wait counters of the exact LZ4F compress kernels (256 x 1 MiB JSON).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r2lz4c_pmc"; mkdir -p "$O"
B="$R/bench.py --workload lz4c --steps 2 --warmup 1 --partitions 256 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA -T -f csv -d "$O/p1" -o c -- python3 $B > "$O/p1.log" 2>&1 || { echo PMC1_FAILED; tail -5 "$O/p1.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES -T -f csv -d "$O/p2" -o c -- python3 $B > "$O/p2.log" 2>&1 || { echo PMC2_FAILED; tail -5 "$O/p2.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum -T -f csv -d "$O/p3" -o c -- python3 $B > "$O/p3.log" 2>&1 || { echo PMC3_FAILED; tail -5 "$O/p3.log"; exit 1; }
python3 "$R/scripts/pmc_table.py" "$O" > "$O/table.txt" 2>&1
grep -A22 "lz4_compress_blocks_kernel" "$O/table.txt"
echo PMC_OK
