# PMC instruction mix of the LZ4F compressor (configs[2] leg).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/c"
B="$R/bench.py --workload lz4c --steps 1 --warmup 0 --partitions 256 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -T -f csv -d "$R/gpurun_out/c/pmc1" -o c -- python3 $B > "$R/gpurun_out/c/pmc1.log" 2>&1 || { echo PMC1_FAILED; tail -5 "$R/gpurun_out/c/pmc1.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS -T -f csv -d "$R/gpurun_out/c/pmc2" -o c -- python3 $B > "$R/gpurun_out/c/pmc2.log" 2>&1 || { echo PMC2_FAILED; exit 1; }
echo PMC_OK
