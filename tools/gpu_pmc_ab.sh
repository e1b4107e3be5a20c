# counter passes over the batched k_linearize for several library builds:
#   tools/gpu_pmc_ab.sh TAG lib1.so lib2.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
i=0
for lib in "$@"; do
  LDSO_BA_LIB=$(realpath $lib) timeout -k 10 600 python tools/pmc_probe.py --kernel k_linearize --out pmc_${TAG}_$i \
   "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
   "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM" \
   "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
   "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
   "TD_BUSY_avr TD_TC_STALL_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
   > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "probe failed"; tail -30 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
  echo "== $lib"; grep "group" gpurun_out/pmc_${TAG}_$i.log
  python -c "
import json; d=json.load(open('gpurun_out/pmc_${TAG}_$i.json'))
for k,v in d.items(): print(k, {a: round(b) for a,b in sorted(v.items())})"
  i=$((i+1))
done
