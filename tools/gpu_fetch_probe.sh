# FETCH_SIZE calibration for k_linearize's 16-B piece gathers (tools/gather_probe_pieces.hip):
# timing, then FETCH_SIZE and the raw TCC_EA0 read-request counters in separate rocprofv3 passes.
# usage: tools/gpu_fetch_probe.sh TAG   -> gpurun_out/fetch_TAG/{timing.log,summary.json}
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fetch_$1
mkdir -p $O
timeout -k 10 120 tools/gather_probe_pieces 1024 > $O/timing.log 2>&1 || { echo "probe failed"; cat $O/timing.log; exit 1; }
cat $O/timing.log
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_pieces -d $GRAFT_REPO_ROOT/$O/fetch -o run --output-format csv -- tools/gather_probe_pieces 1024 > $O/fetch.log 2>&1 || { echo "FETCH_SIZE pass failed"; tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex k_pieces -d $GRAFT_REPO_ROOT/$O/rdreq -o run --output-format csv -- tools/gather_probe_pieces 1024 > $O/rdreq.log 2>&1 || { echo "RDREQ pass failed (counter names?)"; tail -5 $O/rdreq.log; }
python tools/fetch_probe_summary.py $O > $O/summary.json && cat $O/summary.json
echo done
