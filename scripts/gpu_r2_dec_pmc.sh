# Instruction mix of the LZ4F decode kernels (consumer leg, 256 x 1 MiB).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r2dec_pmc"; mkdir -p "$O"
B="$R/bench.py --workload consumer --steps 2 --warmup 1 --partitions 256 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA -T -f csv -d "$O/p1" -o c -- python3 $B > "$O/p1.log" 2>&1 || { echo PMC1_FAILED; tail -5 "$O/p1.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS -T -f csv -d "$O/p2" -o c -- python3 $B > "$O/p2.log" 2>&1 || { echo PMC2_FAILED; tail -5 "$O/p2.log"; exit 1; }
python3 "$R/scripts/pmc_table.py" "$O" > "$O/table.txt" 2>&1
grep -A17 "lz4f_blocks_kernel" "$O/table.txt"
echo PMC_OK
