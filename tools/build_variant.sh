#!/bin/bash
# Build a timing variant of libbanjax_gpu.so with extra compiler flags into
# exp_libs/lib_<name>.so (engine.hip recompiled; the host-only objects reused
# from banjax_amd/build).  Load it with BJX_LIB_PATH=exp_libs/lib_<name>.so.
#   tools/build_variant.sh <name> [-DFLAG ...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p exp_libs/obj
python -c "import banjax_amd.build as b; b.build()"
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable -Wno-unused-result"
hipcc $F "$@" -c -o exp_libs/obj/engine_$name.o banjax_amd/csrc/engine.hip
hipcc $F -shared -o exp_libs/lib_$name.so exp_libs/obj/engine_$name.o banjax_amd/build/regex_compiler.cpp.o \
  banjax_amd/build/tailer.cpp.o banjax_amd/build/node.cpp.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built exp_libs/lib_$name.so"
