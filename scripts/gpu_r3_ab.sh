#!/bin/bash
# A/B of library builds under abtmp/ on one bench workload
#   usage: bash scripts/gpu_r3_ab.sh "lib1 lib2 ..." bench.py-arguments...
set -o pipefail
LIBS="$1"; shift
for l in $LIBS; do
  if [ "$l" = base ]; then unset RDK_HIP_LIB; else export RDK_HIP_LIB="$GRAFT_REPO_ROOT/abtmp/$l"; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-legs "$@" 2>/dev/null | python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$l', d.get('GB_per_s', d.get('value')), 'GB/s ratio', d.get('compression_ratio'), 'kernel_ms', d['roofline']['kernel_ms'])" || exit 1
done
