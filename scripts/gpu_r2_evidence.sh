# Evidence for the current build: per-leg rocprofv3 summaries (trace + HBM counters), instruction-mix
# counters of the exact compressor and the decoder, then the default bench line.
# Copy gpurun_out/prof_r2/summaries/*, gpurun_out/r2lz4c_pmc/table.txt,
# gpurun_out/r2dec_pmc/table.txt and gpurun_out/r2bench/bench.json into profiles/r02/.
set -o pipefail
R="$GRAFT_REPO_ROOT"
bash "$R/scripts/profile_r2_all.sh" || exit 1
bash "$R/scripts/gpu_r2_lz4c_pmc.sh" > "$R/gpurun_out/r2lz4c_pmc.out" 2>&1 || { echo LZ4C_PMC_FAILED; tail -5 "$R/gpurun_out/r2lz4c_pmc.out"; exit 1; }
bash "$R/scripts/gpu_r2_dec_pmc.sh" > "$R/gpurun_out/r2dec_pmc.out" 2>&1 || { echo DEC_PMC_FAILED; tail -5 "$R/gpurun_out/r2dec_pmc.out"; exit 1; }
cd "$R"
O="$R/gpurun_out/r2bench"; mkdir -p "$O"
timeout -k 10 900 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo BENCH_FAILED; tail -30 "$O/bench.err"; exit 1; }
echo EVIDENCE_OK
