// lz4e_results.h -- how the host entry points read a decode batch's return
// values (shared by lz4e_host.hip and the lane emulator's tests).
#pragma once

#include <stdint.h>

#include <string>

namespace lz4e {

// ret[i] of the pipelined decoder when its watchdog fired
// (LZ4E_DECODE_ABORTED of include/lz4e.h; never a reference return value).
constexpr int32_t kDecodeAborted = INT32_MIN;

// Number of blocks with ret >= 0, or -1 (with err set) when the decoder's
// watchdog fired on some block: the call then fails as a whole.
inline int decode_results(const int32_t* ret, uint32_t n, std::string& err) {
    int good = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (ret[i] == kDecodeAborted) {
            err = "lz4e: decoder watchdog fired on block " + std::to_string(i) +
                  " (a wait made no progress; LZ4E_DECODE_ABORTED)";
            return -1;
        }
        if (ret[i] >= 0) good++;
    }
    return good;
}

}  // namespace lz4e
