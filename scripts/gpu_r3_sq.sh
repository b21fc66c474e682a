#!/bin/bash
# SQ occupancy/stall counters of one bench workload, summed per kernel.
#   usage: bash scripts/gpu_r3_sq.sh TAG bench.py-arguments...
set -o pipefail
TAG="$1"; shift
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/sq_$TAG"; rm -rf "$O"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc ${SQ_COUNTERS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS} -T -f csv -d "$O/pmc" -o t -- python3 $R/bench.py --no-cpu-baseline --no-legs --steps 3 --warmup 1 "$@" > "$O/log" 2>&1 || { echo "SQ_FAILED"; tail -5 "$O/log"; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for p in glob.glob(d + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"][:60]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVE_CYCLES":
            cnt[k] += 1
with open(d + "/summary.txt", "w") as f:
    for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:8]:
        line = f"{k} launches={cnt[k]} " + " ".join(f"{n}={v / max(1, cnt[k]):.4g}" for n, v in sorted(c.items()))
        print(line); f.write(line + "\n")
PY
rm -rf "$O/pmc"
