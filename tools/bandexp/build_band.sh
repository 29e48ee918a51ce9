#!/bin/bash
# Builds the band compressor experiment's lane emulator check
# (tools/bandexp/lz4e_band.hip as host C++, 256 threads per workgroup, the
# lane emulator of tools/emu) linked with the oracle:
#   tools/bandexp/build_band.sh OUT_EXE [flags...]   e.g. -fsanitize=address,undefined
set -e
here=$(cd "$(dirname "$0")" && pwd)
csrc="$here/../../lz4-sgori_amd/csrc"
emu="$here/../emu"
out=$1
shift
CXX=${CXX:-/opt/rocm/llvm/bin/clang++}
CC=${CC:-/opt/rocm/llvm/bin/clang}
obj="$out.oracle.o"
$CC -O1 -g "$@" -c "$here/../../oracle/lz4e_oracle.c" -I "$here/../../include" -o "$obj"
$CXX -std=c++20 -O1 -g -pthread -DLZ4E_EMU -I "$emu/include" -I "$here" -I "$csrc" "$@" \
    -x c++ "$emu/emu.cpp" "$here/emu_band.cpp" "$here/emu_band_main.cpp" -x none "$obj" -o "$out"
echo "built $out"
