# A/B (tools/gpu_ab.sh) then PMC groups for one kernel regex on the default build.
# usage: tools/gpu_ab_pmc.sh TAG KERNEL_REGEX name1 name2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; KRX=$2; shift 2
bash tools/gpu_ab.sh $TAG "$@" || exit 1
timeout -k 10 600 python tools/pmc_probe.py --kernel "$KRX" --out pmc_$TAG \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
  "SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM" \
  "FETCH_SIZE" "WRITE_SIZE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TD_TC_STALL_sum" \
  > gpurun_out/pmc_$TAG.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_$TAG.log; exit 1; }
tail -40 gpurun_out/pmc_$TAG.log
