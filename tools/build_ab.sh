# Build experiment variants of libldso_ba.so (LDSO_EXP_* switches in ldso_ba.hip) for tools/ab_libs.py:
#   bash tools/build_ab.sh NAME "-DFLAG=1 ..." [NAME "FLAGS" ...]  ->  abl/NAME/libldso_ba.so
set -e
cd "$(dirname "$0")/../ldso_amd/csrc"
make -s ../lib/ldso_ct.o ../lib/host_math.o
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -Wall -Wno-unused-function -Wno-unused-result -Wno-unused-const-variable"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  out=../../abl/$name; mkdir -p $out
  ( /opt/rocm/bin/hipcc $HIPFLAGS $flags -c -o $out/ldso_ba.o ldso_ba.hip &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libldso_ba.so $out/ldso_ba.o ../lib/ldso_ct.o ../lib/host_math.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib ) &
done
wait
