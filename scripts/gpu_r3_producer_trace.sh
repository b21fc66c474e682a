#!/bin/bash
# kernel + memory-copy timeline of the producer front-end (one thread, 128 MiB slots)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/prod_trace"; rm -rf "$O"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --memory-copy-trace -T -f csv -d "$O/t" -o t -- python3 $R/bench.py --workload producer --partitions 2048 --steps 1 --warmup 0 --no-cpu-baseline --no-legs > "$O/log" 2>&1 || { tail -5 "$O/log"; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
d = sys.argv[1]
ev = []
for p in glob.glob(d + "/t/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K:" + r["Kernel_Name"][:40]))
for p in glob.glob(d + "/t/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C:" + r.get("Direction", "?") ))
ev.sort()
t_end = ev[-1][1]
# last 400 ms of the run: the timed step
tail = [e for e in ev if e[0] > t_end - 120e6]
t0 = tail[0][0]
with open(d + "/timeline.txt", "w") as f:
    for s, e, n in tail:
        if e - s > 20000:
            f.write(f"{(s - t0) / 1e6:9.3f} ms  +{(e - s) / 1e6:7.3f} ms  {n}\n")
def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s_, e_ in iv:
        if cs is None or s_ > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s_, e_
        else:
            ce = max(ce, e_)
    return tot + (ce - cs if cs is not None else 0)
# steady state: the middle 60 % of the last 100 ms
lo, hi = t_end - 80e6, t_end - 20e6
mid = [(max(s_, lo), min(e_, hi), n) for s_, e_, n in ev if e_ > lo and s_ < hi]
span = hi - lo
h2d = [(s_, e_) for s_, e_, n in mid if n.startswith("C:") and e_ - s_ > 100000]
ker = [(s_, e_) for s_, e_, n in mid if n.startswith("K:")]
print(f"steady window {span / 1e6:.1f} ms: bulk H2D engine busy {union(h2d) / span:.2f}, "
      f"any kernel running {union(ker) / span:.2f}, either {union(h2d + ker) / span:.2f}; "
      f"bulk H2D copies {len(h2d)}, sum {sum(e_ - s_ for s_, e_ in h2d) / 1e6:.1f} ms")
import collections
tot = collections.Counter()
for s, e, n in tail:
    tot[n] += e - s
for n, v in tot.most_common(12):
    print(f"{v / 1e6:9.2f} ms  {n}")
print("span ms", (tail[-1][1] - t0) / 1e6)
PY
head -90 "$O/timeline.txt"
rm -rf "$O/t"
