// Standalone check of the emulated band compressor against the oracle:
//   emu_band_main FILE BLOCK_SIZE TABLE_CLASS [NBLOCKS [CAP_DELTA]]
// compresses consecutive blocks of FILE one launch each and compares the
// frame, its size and the iterator post-state words with
// oracle_compress_linear.  CAP_DELTA < 0 makes the output limited.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../oracle/lz4e_oracle.h"

extern "C" int emu_compress_band(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                 const uint8_t* table_type, uint8_t* dst, const uint64_t* dst_off,
                                 const uint32_t* dst_cap, int32_t* ret, uint32_t* aux, uint32_t nblocks,
                                 uint32_t max_len);

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> all;
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) all.insert(all.end(), buf, buf + k);
    fclose(f);
    const uint32_t bs = (uint32_t)atoi(argv[2]);
    const uint8_t tt = (uint8_t)atoi(argv[3]);
    const long nb = argc > 4 ? atol(argv[4]) : 1;
    const int capd = argc > 5 ? atoi(argv[5]) : 0;
    int bad = 0;
    for (long i = 0; i < nb && (size_t)(i + 1) * bs <= all.size(); ++i) {
        std::vector<uint8_t> in(bs ? bs : 1);  // (a valid pointer for an empty block)
        if (bs) memcpy(in.data(), all.data() + i * bs, bs);
        const uint32_t bound = bs + bs / 255 + 16;
        const uint32_t cap = capd < 0 ? (uint32_t)((int)bound + capd) : bound;
        std::vector<uint8_t> out(cap), ref(bound + 64);
        uint64_t so = 0, doff = 0;
        uint32_t len = bs, aux[2] = {7, 7};
        int32_t r = -7;
        emu_compress_band(in.data(), &so, &len, &tt, out.data(), &doff, &cap, &r, aux, 1, bs);
        uint32_t fs = 0, lr = 0;
        const int rr = oracle_compress_linear(in.data(), bs, tt, ref.data(), cap, &fs, &lr);
        const bool ok = r == rr && (rr == 0 || (!memcmp(out.data(), ref.data(), rr) && aux[0] == fs && aux[1] == lr));
        if (!ok) {
            size_t d = 0;
            while (rr > 0 && d < (size_t)rr && out[d] == ref[d]) ++d;
            printf("block %ld: ret %d vs %d, aux %u/%u vs %u/%u, first diff byte %zu\n", i, r, rr, aux[0], aux[1], fs,
                   lr, d);
            if (!bad) {
                FILE* o = fopen("/tmp/emu_band_got.bin", "wb");
                fwrite(out.data(), 1, r > 0 ? r : 0, o);
                fclose(o);
                o = fopen("/tmp/emu_band_want.bin", "wb");
                fwrite(ref.data(), 1, rr > 0 ? rr : 0, o);
                fclose(o);
            }
            ++bad;
        }
    }
    printf("%s bs=%u tt=%u blocks=%ld bad=%d\n", argv[1], bs, tt, nb, bad);
    return bad != 0;
}
