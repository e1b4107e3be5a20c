# Round-2 probe: GPU tests on the current tree + counter passes over the batched k_linearize
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_avail.txt 2>&1 || echo "list failed"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_p0.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_p0.log; exit 1; }
tail -2 gpurun_out/pytest_p0.log
timeout -k 10 900 python tools/pmc_probe.py --kernel k_linearize --out probe_p0 \
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
 "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
 "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_READ_sum TCP_TOTAL_WRITE_sum TCP_TCC_WRITE_REQ_sum" \
 "TD_BUSY_avr TD_TC_STALL_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
 "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_SMEM" \
 > gpurun_out/probe_p0.log 2>&1 || { echo "probe failed"; tail -30 gpurun_out/probe_p0.log; exit 1; }
grep -c "group ok" gpurun_out/probe_p0.log
echo done
