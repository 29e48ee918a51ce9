#!/bin/bash
# Builds the lane emulator: the compress kernel and both decoders (one-wave
# and the 4-wave pipelined one) run on host threads, one per lane, with the
# product's own csrc/lz4e_wave.h (compiled with -DLZ4E_EMU; the amdgcn
# builtins come from tools/emu/include/hip/hip_runtime.h).
#   tools/emu/build.sh [flags...]        -> $EMU_BUILD/libemu.so (default tools/emu/build)
#   EMU_EXE=1 tools/emu/build.sh [flags] -> $EMU_BUILD/emu_main (standalone)
# Pass extra flags, e.g. -fsanitize=address,undefined or -DLZ4E_SPIN_MAX=1.
set -e
here=$(cd "$(dirname "$0")" && pwd)
csrc="$here/../../lz4-sgori_amd/csrc"
b="${EMU_BUILD:-$here/build}"
mkdir -p "$b"
CXX=${CXX:-/opt/rocm/llvm/bin/clang++}
FLAGS=(-std=c++20 -O1 -g -pthread -x c++ -DLZ4E_EMU -I "$here/include" -I "$csrc")
if [ -n "$EMU_EXE" ]; then
    $CXX "${FLAGS[@]}" "$@" "$here/emu.cpp" "$here/emu_dec.cpp" "$here/emu_main.cpp" -o "$b/emu_main"
    echo "built $b/emu_main"
else
    $CXX "${FLAGS[@]}" -fPIC -shared "$@" "$here/emu.cpp" "$here/emu_dec.cpp" -o "$b/libemu.so"
    echo "built $b/libemu.so"
fi
