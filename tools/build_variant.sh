#!/bin/bash
# Build libvbfm.so with extra / different compiler flags into <outdir>/lib for interleaved A/B
# against the product library (VBFM_LIB=<outdir>/lib/libvbfm.so); never the product library.
# usage: tools/build_variant.sh <outdir> [--no-preload] [extra hipcc flags...]
set -e
cd "$(dirname "$0")/.."
P=scalable-variational-bayesian-factorization-machine_amd
O=$1; shift
PRE="-mllvm -amdgpu-kernarg-preload-count=16"
if [ "$1" = "--no-preload" ]; then PRE=""; shift; fi
mkdir -p $O/build $O/lib
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -I/opt/rocm/include $PRE $*"
for s in vbfm_online vbfm_replay vbfm_lorder vbfm_kernels vbfm_mcmc vbfm_capi vbfm_mcmc_capi; do
  /opt/rocm/bin/hipcc $F -c $P/csrc/$s.hip -o $O/build/$s.o &
done
g++ -O2 -std=c++17 -fPIC -ffp-contract=off -Wall -pthread -c $P/csrc/vbfm_host.cpp -o $O/build/vbfm_host.o
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/lib/libvbfm.so $O/build/*.o -L/opt/rocm/lib -lrccl \
  -lrocprofiler-sdk-roctx -pthread -Wl,-rpath,/opt/rocm/lib
echo built $O/lib/libvbfm.so
