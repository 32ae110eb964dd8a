#!/bin/bash
# Build libvbfm.so of a committed tree (default HEAD) into tools/ab_head/lib for interleaved A/B
# against the working tree's product library (VBFM_LIB=tools/ab_head/lib/libvbfm.so).
# usage: tools/build_head.sh [<commit> [<outdir>]]
set -e
cd "$(dirname "$0")/.."
C=${1:-HEAD}
T=$(mktemp -d)
git archive "$C" scalable-variational-bayesian-factorization-machine_amd/csrc include | tar -x -C "$T"
O=${2:-tools/ab_head}
rm -rf $O && mkdir -p $O/build $O/lib
P=$T/scalable-variational-bayesian-factorization-machine_amd
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -I/opt/rocm/include -mllvm -amdgpu-kernarg-preload-count=16"
pids=""
for s in vbfm_online vbfm_replay vbfm_lorder vbfm_kernels vbfm_mcmc vbfm_capi vbfm_mcmc_capi; do
  /opt/rocm/bin/hipcc $F -c $P/csrc/$s.hip -o $O/build/$s.o & pids="$pids $!"
done
g++ -O2 -std=c++17 -fPIC -ffp-contract=off -Wall -pthread -c $P/csrc/vbfm_host.cpp -o $O/build/vbfm_host.o
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o $O/lib/libvbfm.so $O/build/*.o \
  -L/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx -pthread -Wl,-rpath,/opt/rocm/lib
rm -rf "$T"
echo "built $O/lib/libvbfm.so from $(git rev-parse --short $C)"
