set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LDSO_BA_LIN_VARIANT=3 timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_sp.log 2>&1 || { echo "pytest sp failed"; tail -40 gpurun_out/pytest_sp.log; exit 1; }
tail -2 gpurun_out/pytest_sp.log


timeout -k 10 300 python tools/ab_lin.py > gpurun_out/ab_sp.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ab_sp.log; exit 1; }
cat gpurun_out/ab_sp.log
