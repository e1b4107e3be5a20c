#!/bin/bash
# GPU box: tests + bench (tools/gpu_tests_bench.sh), then optional extra steps, each under its own
# time limit; stops at the first abnormal exit (fault / abort / timeout).
# Usage: bash tools/gpu_session.sh TAG [ab LIB1 LIB2 ...] [prof_single] [prof_bench]
TAG=$1; shift
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
bash tools/gpu_tests_bench.sh $TAG --steps 20 --warmup 5; rc=$?
ok $rc || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
while [ $# -gt 0 ]; do
  case $1 in
    ab) shift; libs=""; while [ $# -gt 0 ] && [[ $1 == *.so* ]]; do libs="$libs $1"; shift; done
        timeout -k 10 400 python3 tools/ab_libs.py $libs --rounds 3 > gpurun_out/${TAG}_ab.log 2>&1; rc=$?
        echo "ab rc=$rc"; ok $rc || exit $rc ;;
    prof_single) shift
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_single -o prof -- python3 tools/prof_single.py > gpurun_out/${TAG}_prof_single.log 2>&1; rc=$?
        echo "prof_single rc=$rc"; ok $rc || exit $rc ;;
    prof_bench) shift
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_bench -o prof -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-tracker --no-secondary > gpurun_out/${TAG}_prof_bench.log 2>&1; rc=$?
        echo "prof_bench rc=$rc"; ok $rc || exit $rc ;;
    *) echo "unknown step $1"; exit 2 ;;
  esac
done
