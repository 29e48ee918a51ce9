#!/bin/bash
# Builds the band compressor's lane emulator check (csrc/lz4e_band.hip as
# host C++, 256 threads per workgroup) linked with the oracle:
#   tools/emu/build_band.sh OUT_EXE [flags...]   e.g. -fsanitize=address,undefined
set -e
here=$(cd "$(dirname "$0")" && pwd)
csrc="$here/../../lz4-sgori_amd/csrc"
out=$1
shift
CXX=${CXX:-/opt/rocm/llvm/bin/clang++}
CC=${CC:-/opt/rocm/llvm/bin/clang}
obj="$out.oracle.o"
$CC -O1 -g "$@" -c "$here/../../oracle/lz4e_oracle.c" -I "$here/../../include" -o "$obj"
$CXX -std=c++20 -O1 -g -pthread -DLZ4E_EMU -I "$here/include" -I "$csrc" "$@" \
    -x c++ "$here/emu.cpp" "$here/emu_band.cpp" "$here/emu_band_main.cpp" -x none "$obj" -o "$out"
echo "built $out"
