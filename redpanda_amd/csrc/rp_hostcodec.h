// rp_hostcodec.h — gzip / zstd uncompress on the host (rp_hostcodec.cpp):
// the CPU fallback behind compression::compressor::uncompress.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace rp {
constexpr int kHostGzip = 1, kHostZstd = 4;  // model::compression values
constexpr int kHostCodecError = -1, kHostCodecMissing = -2, kHostCodecOverflow = -3;
// one payload; *out_len = decoded size (also on kHostCodecOverflow)
int host_uncompress(int codec, const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
// compressor::compress for gzip / zstd over frag-byte iobuf fragments (0 =
// one); *out_len = the compressed size (also on kHostCodecOverflow)
int host_compress(int codec, const uint8_t* in, size_t n, size_t frag, uint8_t* out, size_t cap, size_t* out_len);
}  // namespace rp
