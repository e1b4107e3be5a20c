set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
LDSO_BA_LIB=abl/stamps/libldso_ba.so timeout -k 10 200 python tools/solve_stamps.py
