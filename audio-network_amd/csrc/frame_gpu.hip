// frame_gpu.hip — ip.proto framing of decoded symbols on the device (config 5:
// every rank frames its own streams, RCCL gathers frames).
//
// Byte-for-byte the output of demod_frame_symbols (demod_frame.c) applied to
// each stream: symbols packed MSB-first at `bits` per symbol into payloads of
// at most max_payload bytes, each wrapped as a delimited
// ToReceiver{audio_data{opus_encoded_frame = payload}} (ip.proto:32-36,63-65;
// nanopb pb_encode_delimited, network.cpp:389-403). That host codec is pinned
// to the reference's own nanopb (tests/test_frame.py); the GPU tests pin this
// kernel to it.
//
// Grid: one block per (stream, frame); its threads each assemble payload
// bytes from the frame's symbols, thread 0 writes the varint headers.
#include "demod_internal.h"

namespace fskd {

__host__ __device__ inline unsigned varint_len32(unsigned v)
{
    unsigned n = 1;
    while (v >= 0x80) { v >>= 7; ++n; }
    return n;
}

__host__ __device__ inline unsigned frame_bytes(unsigned payload)
{
    const unsigned inner = 1 + varint_len32(payload) + payload;  // AudioData
    const unsigned msg = 1 + varint_len32(inner) + inner;        // ToReceiver
    return varint_len32(msg) + msg;
}

__device__ inline unsigned put_varint32(uint8_t *o, unsigned v)
{
    unsigned n = 0;
    while (v >= 0x80) { o[n++] = (uint8_t)(v | 0x80); v >>= 7; }
    o[n++] = (uint8_t)v;
    return n;
}

struct FrameParams {
    const uint8_t *sym;    // [n_streams][n]
    uint8_t *out;          // [n_streams][stride]
    long long n;           // symbols per stream
    long long stride;      // framed bytes per stream
    unsigned per;          // symbols per full frame
    unsigned full_bytes;   // bytes of one full frame
    int bits;
    int frames;            // frames per stream
};

__global__ __launch_bounds__(256) void frame_streams_kernel(FrameParams p)
{
    const long long s = blockIdx.x / p.frames;
    const int f = (int)(blockIdx.x % p.frames);
    const long long i0 = (long long)f * p.per;
    const long long left = p.n - i0;
    const unsigned cnt = left < (long long)p.per ? (unsigned)left : p.per;
    const unsigned pl = (cnt * (unsigned)p.bits + 7) / 8;
    const uint8_t *sy = p.sym + s * p.n + i0;
    uint8_t *o = p.out + s * p.stride + (long long)f * p.full_bytes;
    const unsigned hdr = frame_bytes(pl) - pl;
    if (threadIdx.x == 0) {
        const unsigned inner = 1 + varint_len32(pl) + pl;
        const unsigned msg = 1 + varint_len32(inner) + inner;
        unsigned q = put_varint32(o, msg);
        o[q++] = 0x0A;  // ToReceiver.audio_data: field 1, wire type 2
        q += put_varint32(o + q, inner);
        o[q++] = 0x0A;  // AudioData.opus_encoded_frame: field 1, wire type 2
        put_varint32(o + q, pl);
    }
    const unsigned mask = (1u << p.bits) - 1u;
    const unsigned total_bits = cnt * (unsigned)p.bits;
    for (unsigned j = threadIdx.x; j < pl; j += blockDim.x) {
        unsigned byte = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const unsigned bp = 8 * j + t;  // bit position in the payload, MSB first
            unsigned bit = 0;
            if (bp < total_bits) {
                const unsigned i = bp / (unsigned)p.bits;
                const unsigned b = (unsigned)p.bits - 1 - bp % (unsigned)p.bits;
                bit = ((sy[i] & mask) >> b) & 1u;
            }
            byte |= bit << (7 - t);
        }
        o[hdr + j] = (uint8_t)byte;
    }
}

long long frame_streams_size(long long n, int bits, long long max_payload, unsigned *per_out,
                             unsigned *full_out, int *frames_out)
{
    const unsigned per = (unsigned)(max_payload * 8 / bits);
    const long long frames = n == 0 ? 0 : (n + per - 1) / per;
    const unsigned full = frame_bytes((per * (unsigned)bits + 7) / 8);
    const long long last_cnt = n - (frames - 1) * (long long)per;
    const long long total =
        frames == 0 ? 0 : (frames - 1) * (long long)full + frame_bytes((unsigned)((last_cnt * bits + 7) / 8));
    if (per_out) *per_out = per;
    if (full_out) *full_out = full;
    if (frames_out) *frames_out = (int)frames;
    return total;
}

hipError_t launch_frame_streams(const uint8_t *d_sym, long long n_streams, long long n, int bits,
                                long long max_payload, uint8_t *d_out, hipStream_t s)
{
    FrameParams p;
    p.sym = d_sym;
    p.out = d_out;
    p.n = n;
    p.bits = bits;
    p.stride = frame_streams_size(n, bits, max_payload, &p.per, &p.full_bytes, &p.frames);
    const long long blocks = n_streams * p.frames;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(frame_streams_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

}  // namespace fskd
