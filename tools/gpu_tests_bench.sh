#!/bin/bash
# GPU box: the -m gpu suite, then (unless a step ended abnormally: fault, abort, timeout) the
# C++ face test and bench.py.  Usage: bash tools/gpu_tests_bench.sh TAG [bench args...]
TAG=${1:-run}
shift
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/${TAG}_gpu_tests.log
tail -3 gpurun_out/${TAG}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal test exit $rc: stopping"; exit $rc; fi
timeout -k 10 400 python bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?
echo "bench rc=$rc"
exit $rc
