// sml_packets.hip — the reference's per-packet PreprocessSingle /
// PostprocessSingle (ppp.cc:69-192, 194-299) for a BURST of packets in one
// launch: what a DPDK worker does between rte_eth_rx_burst and
// rte_eth_tx_burst (dpdk_worker_thread.cc:276-345: PostprocessSingle for
// every received packet, then ReusePacket -> PreprocessSingle of pkt_id + b,
// dpdk_worker_thread_utils.inc:134,177), or an RDMA worker over its
// completions (rdma_worker_thread.cc:244,356).
//
// One wave per packet (a packet is at most 1024 elements = one wave's tile);
// the packet buffers are anywhere the device can address (HBM, or pinned host
// memory such as a NIC's mbuf pool) and are read / written in place:
//   preprocess, packet q:  q >= b: block k = q - b quantized with the scale
//                          of the exponent received for packet k, htonl'd,
//                          the n = min(P, numel - kP) real words written
//                          (the reference leaves the tail of a partial block
//                          stale, ppp.cc:102-109: so do we);
//                          q < B: the exponent of block q into byte 0 of the
//                          extra-info slot (byte 1 untouched, ppp.cc:154)
//   postprocess, packet q: q >= b: block q - b dequantized from the packet
//                          into the slice output (n words);
//                          q < B: the packet's exponent byte kept as block
//                          q's received exponent (ppp.cc:254-260 keeps the
//                          scale; the kernels derive the same scale from it)
// INT32 slices: byte swaps both ways, packet q = block q (ppp.cc:158-190,
// 262-298).  Bit-identical to calling the per-packet entry points in order;
// the only ordering the reference's loop guarantees — packet q + b is
// preprocessed after packet q is postprocessed — is the caller's, across
// bursts (a burst holding both q and q + b is refused).
#include "sml_host.h"

namespace sml {

template <int P, bool RNE>
__global__ __launch_bounds__(kBlockThreads) void k_preprocess_burst(sml_packet_burst a) {
    constexpr int U = P > 256 ? P / 256 : 1;         // 256-element slices per packet
    constexpr int kLanes = P >= 256 ? kWave : P / 4; // lanes holding a slice
    const uint32_t i = blockIdx.x * kWavesPerBlock + wave_index();
    if (i >= a.count) return;
    const int lane = threadIdx.x & (kWave - 1);
    const bool act = lane < kLanes;
    const uint64_t q = a.pkt_ids[i];
    const uint64_t B = (a.numel + P - 1) / P;
    if (a.data_type == SML_INT32) {
        const uint64_t off = q * P, n = a.numel - off < P ? a.numel - off : P;
        const uint32_t* in = reinterpret_cast<const uint32_t*>(a.in) + off;
        uint32_t* dst = static_cast<uint32_t*>(a.entries[i]);
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint64_t j = (uint64_t)u * 256 + lane * 4 + t;
                if (act && j < n) dst[j] = bswap(in[j]);
            }
        return;
    }
    if (q >= a.batch_num_ltus) {
        const uint64_t k = q - a.batch_num_ltus;
        const uint64_t off = k * P, n = a.numel - off < P ? a.numel - off : P;
        const uint64_t body = n / 16 * 16;          // VCL=1: RNE on the 16-aligned body of the block
        const float s = scale_for(a.num_workers, (int)a.recv_exps[k]);
        const float* in = a.in + off;
        uint32_t* dst = static_cast<uint32_t*>(a.entries[i]);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t j = (uint64_t)u * 256 + lane * 4;
            const f4 x = act ? load4_guarded(in + j, j, n) : mkf4(0, 0, 0, 0);
            const u4 w = quantize4<RNE>(x, s, j, body);
            if (act && j + 0 < n) dst[j + 0] = bswap(w.x);
            if (act && j + 1 < n) dst[j + 1] = bswap(w.y);
            if (act && j + 2 < n) dst[j + 2] = bswap(w.z);
            if (act && j + 3 < n) dst[j + 3] = bswap(w.w);
        }
    }
    if (q < B) {
        const uint64_t off = q * P, n = a.numel - off < P ? a.numel - off : P;
        const float* in = a.in + off;
        uint32_t m = 0;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t j = (uint64_t)u * 256 + lane * 4;
            if (act) m = umax(m, max4(load4_guarded(in + j, j, n)));
        }
        m = group_max<256>(m);                     // the wave's max = the packet's (idle lanes hold 0)
        if (lane == 0) *static_cast<int8_t*>(a.extras[i]) = (int8_t)exponent_of(m);
    }
}

template <int P>
__global__ __launch_bounds__(kBlockThreads) void k_postprocess_burst(sml_packet_burst a) {
    constexpr int U = P > 256 ? P / 256 : 1;
    constexpr int kLanes = P >= 256 ? kWave : P / 4;
    const uint32_t i = blockIdx.x * kWavesPerBlock + wave_index();
    if (i >= a.count) return;
    const int lane = threadIdx.x & (kWave - 1);
    const bool act = lane < kLanes;
    const uint64_t q = a.pkt_ids[i];
    const uint64_t B = (a.numel + P - 1) / P;
    const uint32_t* src = static_cast<const uint32_t*>(a.entries[i]);
    if (a.data_type == SML_INT32) {
        const uint64_t off = q * P, n = a.numel - off < P ? a.numel - off : P;
        uint32_t* out = reinterpret_cast<uint32_t*>(a.out) + off;
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint64_t j = (uint64_t)u * 256 + lane * 4 + t;
                if (act && j < n) out[j] = bswap(src[j]);
            }
        return;
    }
    if (q >= a.batch_num_ltus) {
        const uint64_t k = q - a.batch_num_ltus;
        const uint64_t off = k * P, n = a.numel - off < P ? a.numel - off : P;
        const float s = scale_for(a.num_workers, (int)a.recv_exps[k]);
        float* out = a.out + off;
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint64_t j = (uint64_t)u * 256 + lane * 4 + t;
                if (act && j < n) out[j] = dequantize1(bswap(src[j]), s);
            }
    }
    if (q < B && lane == 0) a.recv_exps[q] = *static_cast<const int8_t*>(a.extras[i]);
}

// Host checks shared by both entry points.
static sml_status_t check_burst(const sml_packet_burst* a) {
    if (!a) return SML_ERR_INVALID_ARG;
    if (!valid_packet(a->packet_numel)) return SML_ERR_UNSUPPORTED;
    if (a->count > SML_MAX_BURST || a->num_workers == 0) return SML_ERR_INVALID_ARG;
    if (a->data_type != SML_FLOAT32 && a->data_type != SML_INT32) return SML_ERR_UNSUPPORTED;
    if (a->count == 0) return SML_OK;
    if (!a->in && !a->out) return SML_ERR_INVALID_ARG;
    const uint64_t P = a->packet_numel;
    const uint64_t B = sml_num_blocks(a->numel, (uint32_t)P);
    const bool flt = a->data_type == SML_FLOAT32;
    const uint64_t b = flt ? a->batch_num_ltus : 0;
    if (flt && (!a->recv_exps || b > B)) return SML_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < a->count; i++) {
        const uint64_t q = a->pkt_ids[i];
        if (q >= B + b || !a->entries[i] || (flt && q < B && !a->extras[i])) return SML_ERR_INVALID_ARG;
        for (uint32_t j = 0; j < i; j++)   // distinct, and never q and q + b together
            if (a->pkt_ids[j] == q || (b && (a->pkt_ids[j] == q + b || a->pkt_ids[j] + b == q)))
                return SML_ERR_INVALID_ARG;
    }
    return SML_OK;
}

}  // namespace sml

using namespace sml;

extern "C" {

sml_status_t sml_preprocess_burst(const sml_packet_burst* burst, void* stream) {
    sml_status_t st = check_burst(burst);
    if (st != SML_OK || burst->count == 0) return st;
    if (!burst->in) return SML_ERR_INVALID_ARG;
    const sml_packet_burst& a = *burst;
    const dim3 grid((a.count + kWavesPerBlock - 1) / kWavesPerBlock);
    const hipStream_t s = (hipStream_t)stream;
    const bool rne = (a.flags & SML_FLAG_ROUND_RNE) != 0;
#define SML_PRE(PN)                                                                        \
    if (rne) k_preprocess_burst<PN, true><<<grid, kBlockThreads, 0, s>>>(a);               \
    else k_preprocess_burst<PN, false><<<grid, kBlockThreads, 0, s>>>(a);
    switch (a.packet_numel) {
        case 64: SML_PRE(64) break;
        case 128: SML_PRE(128) break;
        case 256: SML_PRE(256) break;
        case 512: SML_PRE(512) break;
        default: SML_PRE(1024) break;
    }
#undef SML_PRE
    return launch_check();
}

sml_status_t sml_postprocess_burst(const sml_packet_burst* burst, void* stream) {
    sml_status_t st = check_burst(burst);
    if (st != SML_OK || burst->count == 0) return st;
    if (!burst->out) return SML_ERR_INVALID_ARG;
    const sml_packet_burst& a = *burst;
    const dim3 grid((a.count + kWavesPerBlock - 1) / kWavesPerBlock);
    const hipStream_t s = (hipStream_t)stream;
    switch (a.packet_numel) {
        case 64: k_postprocess_burst<64><<<grid, kBlockThreads, 0, s>>>(a); break;
        case 128: k_postprocess_burst<128><<<grid, kBlockThreads, 0, s>>>(a); break;
        case 256: k_postprocess_burst<256><<<grid, kBlockThreads, 0, s>>>(a); break;
        case 512: k_postprocess_burst<512><<<grid, kBlockThreads, 0, s>>>(a); break;
        default: k_postprocess_burst<1024><<<grid, kBlockThreads, 0, s>>>(a); break;
    }
    return launch_check();
}

}  // extern "C"
