#!/bin/bash
# Lab A/B builds: the product library with one translation unit recompiled under
# extra flags -> labbuild/<name>.so.  usage: bash tools/lab_variant.sh <name> <source.hip> <flags...>
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
make -s -C byzantine-agreement_amd
mkdir -p labbuild
B=byzantine-agreement_amd
base=$(basename $src)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall --offload-arch=gfx950 -munsafe-fp-atomics "$@" \
  -c -o labbuild/$name.$base.o $B/csrc/$base
objs=$(ls $B/build/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o labbuild/$name.so \
  $objs labbuild/$name.$base.o -ldl
echo built labbuild/$name.so
