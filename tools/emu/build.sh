#!/bin/bash
# Builds tools/emu/build/libemu.so: the compress kernel source run on host
# threads (one per lane).  Pass extra flags, e.g. -fsanitize=address.
set -e
here=$(cd "$(dirname "$0")" && pwd)
csrc="$here/../../lz4-sgori_amd/csrc"
b="$here/build"
mkdir -p "$b/src"
cp "$csrc"/lz4e_compress.hip "$csrc"/lz4e_device.h "$csrc"/lz4e_gpu.h "$b/src/"
cp "$here/lz4e_wave.h" "$b/src/"
cp "$here/emu.cpp" "$b/src/"
${CXX:-/opt/rocm/llvm/bin/clang++} -std=c++20 -O1 -g -fPIC -shared -pthread -x c++ \
    -I "$here/include" -I "$b/src" "$@" "$b/src/emu.cpp" -o "$b/libemu.so"
echo "built $b/libemu.so"
