# Generic PMC passes over one bench command: bash scripts/gpu_pmc.sh OUTDIR "bench args"
set -o pipefail
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/$1"; mkdir -p "$O"
ARGS="$2"
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU" \
         "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -T -f csv -d "$O/p$i" -o p -- python3 $R/bench.py $ARGS > "$O/p$i.log" 2>&1 || { echo "PMC$i FAILED: $P"; tail -5 "$O/p$i.log"; exit 1; }
done
echo PMC_OK
