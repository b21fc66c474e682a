#!/bin/bash
# L1 / L2 hit counters of one bench workload, summed per kernel.
#   usage: bash scripts/gpu_r3_cache.sh TAG bench.py-arguments...
set -o pipefail
TAG="$1"; shift
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/cache_$TAG"; rm -rf "$O"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum -T -f csv -d "$O/pmc" -o t -- python3 $R/bench.py --no-cpu-baseline --no-legs --steps 3 --warmup 1 "$@" > "$O/log" 2>&1 || { echo "PMC_FAILED"; tail -5 "$O/log"; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for p in glob.glob(d + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"][:50]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "TCC_REQ_sum":
            cnt[k] += 1
for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("TCC_REQ_sum", 0))[:4]:
    print(k, f"launches={cnt[k]}", " ".join(f"{n}={v / max(1, cnt[k]):.4g}" for n, v in sorted(c.items())))
PY
rm -rf "$O/pmc"
