// Standalone driver of the lane emulator (sanitizer runs, debuggers):
//   emu_main BLOCK_FILE TABLE_CLASS [FRAME_OUT [DICT_FILE]]
//   emu_main -d FRAME_FILE CAPACITY [OUT_FILE [DICT_FILE]]   (one-wave decoder)
//   emu_main -p FRAME_FILE CAPACITY [OUT_FILE [DICT_FILE]]   (pipelined decoder,
//            4 waves: parser + 3 copiers)
//   emu_main -l FRAME_FILE CAPACITY [OUT_FILE [DICT_FILE]]   (one-wave decoder,
//            LDS output for blocks of <= 4608 bytes without a dictionary)
//   emu_main -g FRAME_FILE CAPACITY [OUT_FILE [DICT_FILE]]   (block-per-group
//            decoder, 8 lanes a block)
//   emu_main -G FRAME_FILE CAPACITY [OUT_FILE [DICT_FILE]]   (the same without
//            the hand-over: every block decoded to its end by its group)
// compresses one block through the unmodified kernel source, prints the
// return value and the iterator post-state words, and writes the frame.
// With DICT_FILE the block is compressed in dictionary mode against the
// file's last <= 64 KiB (staged right before the block, as the library does).
// Buffers are sized exactly (no slack) so that ASan sees any overrun.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

extern "C" int emu_compress_batch(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                  const uint8_t* table_type, uint8_t* dst, const uint64_t* dst_off,
                                  const uint32_t* dst_cap, int32_t* ret, uint32_t* aux,
                                  uint32_t nblocks, uint32_t max_len);
extern "C" int emu_compress_batch_dict(const uint8_t* src, const uint64_t* src_off,
                                       const uint32_t* src_len, const uint8_t* table_type,
                                       uint8_t* dst, const uint64_t* dst_off, const uint32_t* dst_cap,
                                       int32_t* ret, uint32_t* aux, uint32_t nblocks, uint32_t max_len,
                                       const uint32_t* dict_len);

static std::vector<uint8_t> slurp(const char* path) {
    std::vector<uint8_t> v;
    FILE* f = fopen(path, "rb");
    if (!f) exit(2);
    int c;
    while ((c = fgetc(f)) != EOF) v.push_back((uint8_t)c);
    fclose(f);
    return v;
}

extern "C" int emu_decode_results(const int32_t* ret, uint32_t n, char* err, uint32_t err_cap);
extern "C" int emu_decompress_batch_mode(const uint8_t* src, const uint64_t* src_off,
                                         const int32_t* src_len, uint8_t* dst, const uint64_t* dst_off,
                                         const int32_t* dst_cap, int32_t* ret, uint32_t nblocks,
                                         const int32_t* dict_len, uint32_t mode);

// Decode: the frame in an exactly sized buffer, the output buffer exactly
// [dictionary (last <= 64 KiB) | capacity] -- ASan sees any read before the
// dictionary or any write past the capacity.
static int decode_main(int argc, char** argv) {
    std::vector<uint8_t> frame = slurp(argv[2]);
    const int32_t cap = atoi(argv[3]);
    std::vector<uint8_t> dict;
    if (argc > 5) dict = slurp(argv[5]);
    const int32_t D = (int32_t)(dict.size() > 65536 ? 65536 : dict.size());
    std::vector<uint8_t> out(dict.end() - D, dict.end());
    out.resize((size_t)D + (size_t)cap);
    const int32_t csize = (int32_t)frame.size();
    const uint64_t so = 0, doff = (uint64_t)D;
    int32_t ret = -7777;
    if (frame.empty()) frame.push_back(0);  // a valid pointer for csize 0
    // the decoder reads the input window by aligned dwords (the GPU's word
    // granularity: the dword holding the last byte); the heap block covers it
    frame.reserve((frame.size() + 3) & ~(size_t)3);
    // kDecPipe / kDecSmall / kDecGroup / kDecWave
    const char m = argv[1][1];
    const uint32_t mode = m == 'p' ? 2u : (m == 'l' ? 6u : (m == 'g' ? 7u : (m == 'G' ? 9u : 1u)));
    emu_decompress_batch_mode(frame.data(), &so, &csize, out.data(), &doff, &cap, &ret, 1, &D, mode);
    char err[256];
    const int good = emu_decode_results(&ret, 1, err, sizeof err);
    printf("ret %d\nresults %d %s\n", ret, good, err);
    if (argc > 4 && ret > 0) {
        FILE* o = fopen(argv[4], "wb");
        if (!o) return 2;
        fwrite(out.data() + D, 1, (size_t)ret, o);
        fclose(o);
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 3 && argv[1][0] == '-' &&
        (argv[1][1] == 'd' || argv[1][1] == 'p' || argv[1][1] == 'l' || argv[1][1] == 'g' || argv[1][1] == 'G'))
        return decode_main(argc, argv);
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
    std::vector<uint8_t> dict;
    if (argc > 4) dict = slurp(argv[4]);
    uint32_t D = (uint32_t)dict.size() > 65536 ? 65536 : (uint32_t)dict.size();
    std::vector<uint8_t> src(dict.end() - D, dict.end()), dst(cap);
    src.insert(src.end(), in.begin(), in.end());
    const uint64_t so = D, doff = 0;
    int32_t ret = -7;
    uint32_t aux[2] = {0, 0};
    if (argc > 4)
        emu_compress_batch_dict(src.data(), &so, &n, &tt, dst.data(), &doff, &cap, &ret, aux, 1, n, &D);
    else
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
