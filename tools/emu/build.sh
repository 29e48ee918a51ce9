#!/bin/bash
# Builds the lane emulator: the compress kernel and the one-wave decoder
# sources run on host threads (one per lane).
#   tools/emu/build.sh [flags...]        -> tools/emu/build/libemu.so
#   EMU_EXE=1 tools/emu/build.sh [flags] -> tools/emu/build/emu_main (standalone)
# Pass extra flags, e.g. -fsanitize=address,undefined.
set -e
here=$(cd "$(dirname "$0")" && pwd)
csrc="$here/../../lz4-sgori_amd/csrc"
b="${EMU_BUILD:-$here/build}"
mkdir -p "$b/src"
cp "$csrc"/lz4e_compress.hip "$csrc"/lz4e_decompress.hip "$csrc"/lz4e_device.h "$csrc"/lz4e_gpu.h "$csrc"/lz4e_order.h "$b/src/"
cp "$here/lz4e_wave.h" "$b/src/"
cp "$here/emu.cpp" "$here/emu_dec.cpp" "$b/src/"
CXX=${CXX:-/opt/rocm/llvm/bin/clang++}
if [ -n "$EMU_EXE" ]; then
    $CXX -std=c++20 -O1 -g -pthread -x c++ -I "$here/include" -I "$b/src" "$@" \
        "$b/src/emu.cpp" "$b/src/emu_dec.cpp" "$here/emu_main.cpp" -o "$b/emu_main"
    echo "built $b/emu_main"
else
    $CXX -std=c++20 -O1 -g -fPIC -shared -pthread -x c++ \
        -I "$here/include" -I "$b/src" "$@" "$b/src/emu.cpp" "$b/src/emu_dec.cpp" -o "$b/libemu.so"
    echo "built $b/libemu.so"
fi
