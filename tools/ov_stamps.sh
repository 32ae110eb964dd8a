#!/bin/bash
# Diagnostic build of libvbfm.so with per-workgroup phase stamps in the online level kernel
# (k_ov_lord, -DVBFM_OV_STAMPS) into tools/ab_stamp/lib/libvbfm.so; never the product library.
# Run: VBFM_LIB=tools/ab_stamp/lib/libvbfm.so VBFM_OV_STAMP=<launch> python bench.py --config c3 --method vb_online ...
set -e
cd "$(dirname "$0")/.."
P=scalable-variational-bayesian-factorization-machine_amd
O=tools/ab_stamp
mkdir -p $O/build $O/lib
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -I/opt/rocm/include -DVBFM_OV_STAMPS"
for s in vbfm_online vbfm_replay vbfm_lorder vbfm_kernels vbfm_mcmc vbfm_capi vbfm_mcmc_capi; do
  /opt/rocm/bin/hipcc $F -c $P/csrc/$s.hip -o $O/build/$s.o &
done
g++ -O2 -std=c++17 -fPIC -ffp-contract=off -Wall -pthread -c $P/csrc/vbfm_host.cpp -o $O/build/vbfm_host.o
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/lib/libvbfm.so $O/build/*.o -L/opt/rocm/lib -lrccl \
  -lrocprofiler-sdk-roctx -pthread -Wl,-rpath,/opt/rocm/lib
echo built $O/lib/libvbfm.so
