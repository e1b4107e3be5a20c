# SQ/TA counter probe of the bench kernels + k_linearize split (accumulate on/off)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_lin.py > gpurun_out/ab_probe.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ab_probe.log; exit 1; }
cat gpurun_out/ab_probe.log
timeout -k 10 900 python tools/pmc_probe.py "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" > gpurun_out/probe.log 2>&1 || { echo "probe failed"; tail -30 gpurun_out/probe.log; exit 1; }
tail -5 gpurun_out/probe.log
