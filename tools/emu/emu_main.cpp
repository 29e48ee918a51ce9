// Standalone driver of the lane emulator (sanitizer runs, debuggers):
//   emu_main BLOCK_FILE TABLE_CLASS [FRAME_OUT]
// compresses one block through the unmodified kernel source, prints the
// return value and the iterator post-state words, and writes the frame.
// Buffers are sized exactly (no slack) so that ASan sees any overrun.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

extern "C" int emu_compress_batch(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                  const uint8_t* table_type, uint8_t* dst, const uint64_t* dst_off,
                                  const uint32_t* dst_cap, int32_t* ret, uint32_t* aux,
                                  uint32_t nblocks, uint32_t max_len);

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: emu_main BLOCK_FILE TABLE_CLASS [FRAME_OUT]\n");
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> in;
    int c;
    while ((c = fgetc(f)) != EOF) in.push_back((uint8_t)c);
    fclose(f);
    const uint32_t n = (uint32_t)in.size();
    const uint8_t tt = (uint8_t)atoi(argv[2]);
    const uint32_t cap = n + n / 255 + 16;
    std::vector<uint8_t> src(in), dst(cap);
    const uint64_t so = 0, doff = 0;
    int32_t ret = -7;
    uint32_t aux[2] = {0, 0};
    emu_compress_batch(src.data(), &so, &n, &tt, dst.data(), &doff, &cap, &ret, aux, 1, n);
    printf("ret %d aux %u %u\n", ret, aux[0], aux[1]);
    if (argc > 3 && ret > 0) {
        FILE* o = fopen(argv[3], "wb");
        if (!o) return 2;
        fwrite(dst.data(), 1, (size_t)ret, o);
        fclose(o);
    }
    return 0;
}
