#!/bin/bash
# threaded drop-in test, host-path tests, then the drop-in bench leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_threads.py tests/test_gpu_host_paths.py tests/test_gpu_errors.py tests/test_gpu_interpose.py -x -v --timeout 180 --timeout-method thread > gpurun_out/threads_test.log 2>&1
rc=$?
tail -15 gpurun_out/threads_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload dropin > gpurun_out/dropin.json 2> gpurun_out/dropin.err || { tail -5 gpurun_out/dropin.err; exit 1; }
RDK_HIP_COMBINE=0 timeout -k 10 300 python -u bench.py --workload dropin --no-cpu-baseline > gpurun_out/dropin_uncombined.json 2> gpurun_out/dropin_uncombined.err || { tail -5 gpurun_out/dropin_uncombined.err; exit 1; }
RDK_HIP_COMBINE_WAIT_US=0 timeout -k 10 300 python -u bench.py --workload dropin --no-cpu-baseline > gpurun_out/dropin_nowait.json 2> gpurun_out/dropin_nowait.err || { tail -5 gpurun_out/dropin_nowait.err; exit 1; }
echo done
