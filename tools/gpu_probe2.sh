set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python tools/pmc_probe.py "FETCH_SIZE" "TCP_TCC_READ_REQ_sum" "TCP_TOTAL_CACHE_ACCESSES_sum" "TA_BUSY_avr" "TCC_BUSY_avr" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD" > gpurun_out/probe2.log 2>&1 || { echo "probe failed"; tail -30 gpurun_out/probe2.log; exit 1; }
grep "group failed" gpurun_out/probe2.log || true
python -c "
import json; d=json.load(open('gpurun_out/pmcprobe.json'))
for k in d:
    print(k, {c: round(v) for c, v in d[k].items()})
"
