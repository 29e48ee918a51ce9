#!/bin/bash
# Builds a decoder variant of the library: lz4-sgori_amd/build/var/lib<NAME>.so
# with lz4e_decompress.hip compiled with the extra flags (the default compress
# and host objects).  usage: tools/build_decvar.sh NAME [-DFLAG=...]...
set -e
cd "$(dirname "$0")/../lz4-sgori_amd"
name=$1; shift
mkdir -p build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" \
    -c csrc/lz4e_decompress.hip -o build/var/dec_$name.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build/var/lib$name.so \
    build/lz4e_compress.o build/var/dec_$name.o build/lz4e_host.o
echo built build/var/lib$name.so
