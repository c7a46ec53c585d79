#!/bin/bash
# Lab build: libba_hip with the units kernel's per-wave phase stamps
# (ba_cascade.hip, -DBA_CASC_STAMPS) -> labbuild/libba_hip_stamps.so, linked from
# the product objects plus a stamped ba_cascade.hip.o.  Run on it:
#   BA_HIP_LIB=$PWD/labbuild/libba_hip_stamps.so python tools/casc_stamps.py --batch 1024
set -e
cd "$(dirname "$0")/.."
make -s -C byzantine-agreement_amd
mkdir -p labbuild
B=byzantine-agreement_amd
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall --offload-arch=gfx950 -munsafe-fp-atomics \
  -DBA_CASC_STAMPS -c -o labbuild/ba_cascade_stamps.o $B/csrc/ba_cascade.hip
objs=$(ls $B/build/*.o | grep -v ba_cascade.hip.o)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o labbuild/libba_hip_stamps.so \
  $objs labbuild/ba_cascade_stamps.o -ldl
echo built labbuild/libba_hip_stamps.so
