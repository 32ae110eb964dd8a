#!/bin/bash
# Build a libvbfm.so WITHOUT the barriers that separate the waves' reads of a column's old
# parameter from the write of its new value in the split forms (the lines tagged [raw-barrier]:
# the round-5 race fix) into <outdir>/lib, from a copy of csrc/ -- never the product library.
# tests/test_skew_gpu.py must FAIL against it under VBFM_DEBUG_SKEW=1 (and pass on the product):
#   VBFM_LIB=<outdir>/lib/libvbfm.so python -m pytest tests/test_skew_gpu.py -m gpu
# usage: tools/build_nobarrier.sh <outdir>
set -e
cd "$(dirname "$0")/.."
P=scalable-variational-bayesian-factorization-machine_amd
O=$(realpath -m "$1")
mkdir -p $O/build $O/lib $O/src/csrc $O/include
cp $P/csrc/* $O/src/csrc/
cp include/vbfm.h $O/include/
sed -i '/\[raw-barrier\]/d' $O/src/csrc/*.hip
n=$(grep -c "raw-barrier" $P/csrc/*.hip | awk -F: '{s+=$2} END {print s}')
echo "dropped $n barriers"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -I/opt/rocm/include -mllvm -amdgpu-kernarg-preload-count=16"
# the sources include ../../include/vbfm.h: src/csrc -> include/ one level above src
rm -f $O/build/*.o $O/lib/libvbfm.so
pids=()
for s in vbfm_online vbfm_replay vbfm_lorder vbfm_kernels vbfm_mcmc vbfm_capi vbfm_mcmc_capi; do
  /opt/rocm/bin/hipcc $F -c $O/src/csrc/$s.hip -o $O/build/$s.o &
  pids+=($!)
done
g++ -O2 -std=c++17 -fPIC -ffp-contract=off -Wall -pthread -c $O/src/csrc/vbfm_host.cpp -o $O/build/vbfm_host.o
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/lib/libvbfm.so $O/build/*.o -L/opt/rocm/lib -lrccl \
  -lrocprofiler-sdk-roctx -pthread -Wl,-rpath,/opt/rocm/lib
echo built $O/lib/libvbfm.so
