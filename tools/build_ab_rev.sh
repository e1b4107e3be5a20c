# Build libldso_ba.so from ldso_ba.hip as of a git revision (the other sources from the tree):
#   bash tools/build_ab_rev.sh NAME REV  ->  abl/NAME/libldso_ba.so
set -e
cd "$(dirname "$0")/../ldso_amd/csrc"
make -s ../lib/ldso_ct.o ../lib/host_math.o
name=$1; rev=$2; out=../../abl/$name; mkdir -p $out
git show $rev:ldso_amd/csrc/ldso_ba.hip > ldso_ba_rev_tmp.hip
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -Wall -Wno-unused-function -Wno-unused-result -Wno-unused-const-variable"
/opt/rocm/bin/hipcc $HIPFLAGS -c -o $out/ldso_ba.o ldso_ba_rev_tmp.hip && rm -f ldso_ba_rev_tmp.hip
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libldso_ba.so $out/ldso_ba.o ../lib/ldso_ct.o ../lib/host_math.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
