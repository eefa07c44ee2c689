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
// bursts (a burst holding both q and q + b is refused), or the exchange
// burst's, which does both for a received packet in one wave (post of q,
// then pre of q + b into the same buffer: one launch per rx burst).
#include <algorithm>
#include <chrono>

#include "sml_host.h"

namespace sml {

template <int P, bool RNE>
__device__ __forceinline__ void preprocess_one(const sml_packet_burst& a, uint32_t i) {
    constexpr int U = P > 256 ? P / 256 : 1;         // 256-element slices per packet
    constexpr int kLanes = P >= 256 ? kWave : P / 4; // lanes holding a slice
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
            if (act && j + 4 <= n) {
                *reinterpret_cast<u4a*>(dst + j) = u4a{bswap(w.x), bswap(w.y), bswap(w.z), bswap(w.w)};
            } else {
                if (act && j + 0 < n) dst[j + 0] = bswap(w.x);
                if (act && j + 1 < n) dst[j + 1] = bswap(w.y);
                if (act && j + 2 < n) dst[j + 2] = bswap(w.z);
                if (act && j + 3 < n) dst[j + 3] = bswap(w.w);
            }
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
__device__ __forceinline__ void postprocess_one(const sml_packet_burst& a, uint32_t i) {
    constexpr int U = P > 256 ? P / 256 : 1;
    constexpr int kLanes = P >= 256 ? kWave : P / 4;
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
        for (int u = 0; u < U; u++) {
            const uint64_t j = (uint64_t)u * 256 + lane * 4;
            if (act && j + 4 <= n) {   // one 16-B read of the packet per lane
                const u4a v = *reinterpret_cast<const u4a*>(src + j);
                const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int t = 0; t < 4; t++) out[j + t] = dequantize1(bswap(vv[t]), s);
            } else {
#pragma unroll
                for (int t = 0; t < 4; t++)
                    if (act && j + t < n) out[j + t] = dequantize1(bswap(src[j + t]), s);
            }
        }
    }
    if (q < B && lane == 0) a.recv_exps[q] = *static_cast<const int8_t*>(a.extras[i]);
}

// One wave per RECEIVED packet q, the DPDK receive loop's two calls on one
// mbuf in one launch (dpdk_worker_thread.cc:300-345: PostprocessSingle of the
// packet, then ReusePacket -> PreprocessSingle of pkt_id + b into the same
// buffer, dpdk_worker_thread_utils.inc:134,177), optionally preceded by the
// dummy backend's ProcessPacket (x W on all P words, dummy_backend.cc:72-84):
//   FLOAT32  post: q >= b: block q - b dequantized with recv_exps[q - b];
//                  q < B: the packet's exponent byte -> recv_exps[q]
//            pre (q < B, i.e. q + b < B + b): block q quantized with that same
//                  received exponent (its n real words; a partial block's tail
//                  keeps the packet's words), exponent of block q + b into
//                  byte 0 of the extra slot when q + b < B
//   INT32    post: block q byte-swapped into out; pre (q + b < B): block q + b
//                  byte-swapped into the buffer (b = the packet window)
// Every load of the packet is waited for before its buffer is written: the
// reads and the writes of one buffer may cross PCIe (pinned mbufs), where a
// posted write may overtake an outstanding read.
template <int P, bool RNE, bool PROC>
__device__ __forceinline__ void exchange_one(const sml_packet_burst& a, uint32_t i) {
    constexpr int U = P > 256 ? P / 256 : 1;
    constexpr int kLanes = P >= 256 ? kWave : P / 4;
    const int lane = threadIdx.x & (kWave - 1);
    const bool act = lane < kLanes;
    const uint64_t q = a.pkt_ids[i];
    const uint64_t B = (a.numel + P - 1) / P;
    const uint64_t b = a.batch_num_ltus;
    const bool flt = a.data_type == SML_FLOAT32;
    auto real = [&](uint64_t k) -> uint64_t { return a.numel - k * P < P ? a.numel - k * P : P; };
    uint32_t* ent = static_cast<uint32_t*>(a.entries[i]);
    const int8_t* ext = static_cast<const int8_t*>(a.extras[i]);

    // what each half touches: post reads words [0, n_post) of the packet
    // (all P under PROC), pre rewrites words [0, n_pre)
    const bool post_pay = flt ? q >= b : true;
    const uint64_t n_post = !post_pay ? 0 : real(flt ? q - b : q);
    const bool pre = flt ? q < B : q + b < B;
    const uint64_t n_pre = !pre ? 0 : real(flt ? q : q + b);
    const bool pre_exp = flt && q + b < B;
    const uint64_t n_read = PROC ? P : n_post;

    // ---- every load up front
    uint32_t w[U][4];
    f4 xq[U], xe[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        {   // one 16-B access per lane where the group is whole (a packet over
            // PCIe then costs one read per 64 B line, not four)
            const uint64_t j = (uint64_t)u * 256 + lane * 4;
            if (act && j + 4 <= n_read) {
                const u4a v = *reinterpret_cast<const u4a*>(ent + j);
                w[u][0] = v.x, w[u][1] = v.y, w[u][2] = v.z, w[u][3] = v.w;
            } else {
#pragma unroll
                for (int t = 0; t < 4; t++) w[u][t] = act && j + t < n_read ? ent[j + t] : 0u;
            }
        }
        const uint64_t j = (uint64_t)u * 256 + lane * 4;
        if (flt) {
            xq[u] = act && pre ? load4_guarded(a.in + q * P + j, j, n_pre) : mkf4(0, 0, 0, 0);
            xe[u] = act && pre_exp ? load4_guarded(a.in + (q + b) * P + j, j, real(q + b)) : mkf4(0, 0, 0, 0);
        } else {
            const float* src = a.in + (q + b) * P + j;   // int32 words, read as raw bits
            xq[u] = act && pre ? load4_guarded(src, j, n_pre) : mkf4(0, 0, 0, 0);
        }
    }
    const int e_recv = flt && q < B ? (int)*ext : 0;     // the packet's (aggregated) exponent byte
    const int e_post = flt && q >= b ? (int)a.recv_exps[q - b] : 0;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

    // ---- ProcessPacket, postprocess
    const uint32_t W = a.num_workers;
    if constexpr (PROC) {
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int t = 0; t < 4; t++) w[u][t] = bswap(bswap(w[u][t]) * W);
    }
    if (post_pay) {
        const uint64_t k = flt ? q - b : q;
        const float s = flt ? scale_for(W, e_post) : 0.0f;
        uint32_t* out = reinterpret_cast<uint32_t*>(a.out) + k * P;
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint64_t j = (uint64_t)u * 256 + lane * 4 + t;
                if (act && j < n_post)
                    out[j] = flt ? __float_as_uint(dequantize1(bswap(w[u][t]), s)) : bswap(w[u][t]);
            }
    }
    if (flt && q < B && lane == 0) a.recv_exps[q] = (int8_t)e_recv;

    // ---- preprocess of q + b into the same buffer
    if (pre) {
        const float s = flt ? scale_for(W, e_recv) : 0.0f;
        const uint64_t body = n_pre / 16 * 16;              // VCL=1: RNE on the 16-aligned body
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t j = (uint64_t)u * 256 + lane * 4;
            u4 v;
            if (flt) {
                v = quantize4<RNE>(xq[u], s, j, body);
            } else {
                v = mku4(__float_as_uint(xq[u].x), __float_as_uint(xq[u].y), __float_as_uint(xq[u].z),
                         __float_as_uint(xq[u].w));
            }
            const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int t = 0; t < 4; t++)
                if (act && j + t < n_pre) w[u][t] = bswap(vv[t]);
        }
    }
    // the buffer's words: the new packet's, or (PROC) the processed ones
    const uint64_t n_write = PROC ? P : n_pre;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t j = (uint64_t)u * 256 + lane * 4;
        if (act && j + 4 <= n_write) {
            *reinterpret_cast<u4a*>(ent + j) = u4a{w[u][0], w[u][1], w[u][2], w[u][3]};
        } else {
#pragma unroll
            for (int t = 0; t < 4; t++)
                if (act && j + t < n_write) ent[j + t] = w[u][t];
        }
    }
    if (pre_exp) {
        uint32_t m = 0;
#pragma unroll
        for (int u = 0; u < U; u++) m = umax(m, max4(xe[u]));
        m = group_max<256>(m);                              // idle lanes hold 0
        if (lane == 0) *static_cast<int8_t*>(a.extras[i]) = (int8_t)exponent_of(m);
    }
}

// One launch per burst: a wave per packet.
template <int P, bool RNE>
__global__ __launch_bounds__(kBlockThreads) void k_preprocess_burst(sml_packet_burst a) {
    const uint32_t i = blockIdx.x * kWavesPerBlock + wave_index();
    if (i < a.count) preprocess_one<P, RNE>(a, i);
}

template <int P>
__global__ __launch_bounds__(kBlockThreads) void k_postprocess_burst(sml_packet_burst a) {
    const uint32_t i = blockIdx.x * kWavesPerBlock + wave_index();
    if (i < a.count) postprocess_one<P>(a, i);
}

template <int P, bool RNE, bool PROC>
__global__ __launch_bounds__(kBlockThreads) void k_exchange_burst(sml_packet_burst a) {
    const uint32_t i = blockIdx.x * kWavesPerBlock + wave_index();
    if (i < a.count) exchange_one<P, RNE, PROC>(a, i);
}

// ---- the persistent burst server (include/switchml_hip.h) ----------------
// kServerGroups resident workgroups of 16 waves — one wave per packet of a
// full burst — poll a doorbell in coherent, device-mapped host memory.  Per
// burst, in every workgroup: thread 0 polls the doorbell with relaxed
// system-scope loads and, once it moves, acquires at system scope (no stale
// copy of the host-written descriptor or packets); a barrier orders the other
// threads after it; the descriptor is copied into LDS with system-scope
// loads; the waves run their packets (the same per-packet bodies as the
// one-launch-per-burst kernels); a barrier orders every wave's stores before
// thread 0, which releases them at system scope and arrives on a counter in
// device memory.  The last workgroup to arrive resets the counter and
// publishes the burst's sequence number with a system-scope release store;
// the host submits the next burst only after that, so no workgroup can run
// ahead into the next burst.  The loop ends on `stop` or after idle_ticks of
// wall clock without a doorbell, so every wave reaches the exit on its own;
// the host restarts a server that has been idle for half that long before
// ringing it again, so a doorbell never races an idle exit.
constexpr int kServerThreads = 1024;
constexpr int kServerGroups = SML_MAX_BURST / (kServerThreads / kWave);   // 4

struct alignas(64) ServerCtl {
    uint64_t doorbell;         // host: (sequence number << 2) | SML_BURST_* of the last submitted burst
    uint32_t stop;             // host: 1 = leave the loop
    uint32_t pad_stop;
    uint64_t pad0[6];
    uint64_t done;             // device: sequence number of the last completed burst
    uint32_t exited[kServerGroups];   // device: workgroup g has left its loop
    uint64_t pad2[5];
    sml_packet_burst burst;    // host: the submitted burst
};

// A system-scope load without acquire semantics: polling must not invalidate
// the caches on every probe (an acquire load does); the one acquire fence
// follows the probe that sees the doorbell.
template <class T>
__device__ __forceinline__ T sys_poll(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int P, bool RNE>
__global__ __launch_bounds__(kServerThreads) void k_burst_server(ServerCtl* ctl, uint32_t* arrive,
                                                                 uint64_t idle_ticks) {
    __shared__ sml_packet_burst sa;
    __shared__ uint64_t s_seq;
    __shared__ int s_cmd;
    constexpr uint32_t kWaves = kServerThreads / kWave;
    constexpr uint32_t kAllWaves = kWaves * kServerGroups;
    const uint32_t tid = threadIdx.x;
    uint64_t seen = tid == 0 ? sys_poll(&ctl->done) : 0;
    for (;;) {
        if (tid == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            int cmd = -1;
            uint64_t db = seen;
            for (;;) {
                if (sys_poll(&ctl->stop)) break;
                db = sys_poll(&ctl->doorbell) >> 2;
                if (db != seen) {
                    // acquire once, by the thread that saw the doorbell; the
                    // barrier below orders every other thread after it.  The
                    // op rides in the doorbell word (no second round trip).
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                    cmd = (int)(sys_poll(&ctl->doorbell) & 3u);
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) break;
                __builtin_amdgcn_s_sleep(2);
            }
            s_cmd = cmd;
            s_seq = db;
        }
        __syncthreads();
        const int cmd = s_cmd;
        if (cmd < 0) break;
        static_assert(sizeof(sml_packet_burst) % 8 == 0, "descriptor copied in 8-byte words");
        constexpr uint32_t kWords = sizeof(sml_packet_burst) / 8;
        const uint64_t* src = reinterpret_cast<const uint64_t*>(&ctl->burst);
        uint64_t* dst = reinterpret_cast<uint64_t*>(&sa);
        for (uint32_t k = tid; k < kWords; k += kServerThreads)
            dst[k] = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __syncthreads();
        const uint32_t n = sa.count;
        const bool proc = (sa.flags & SML_FLAG_PROCESS_PACKET) != 0;
        for (uint32_t i = blockIdx.x * kWaves + wave_index(); i < n; i += kAllWaves) {
            if (cmd == SML_BURST_PRE) preprocess_one<P, RNE>(sa, i);
            else if (cmd == SML_BURST_POST) postprocess_one<P>(sa, i);
            else if (proc) exchange_one<P, RNE, true>(sa, i);
            else exchange_one<P, RNE, false>(sa, i);
        }
        __syncthreads();
        if (tid == 0) {
            seen = s_seq;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // this workgroup's stores, system-wide
            const uint32_t before = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (before == kServerGroups - 1) {              // the last one: every group's stores are released
                __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&ctl->done, seen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    if (tid == 0) __hip_atomic_store(&ctl->exited[blockIdx.x], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Host checks shared by the entry points.  `window`: the exchange burst's
// packet window b applies to INT32 slices too (the next packet is q + b).
static sml_status_t check_burst(const sml_packet_burst* a, bool window = false) {
    if (!a) return SML_ERR_INVALID_ARG;
    if (!valid_packet(a->packet_numel)) return SML_ERR_UNSUPPORTED;
    if (a->count > SML_MAX_BURST || a->num_workers == 0) return SML_ERR_INVALID_ARG;
    if (a->data_type != SML_FLOAT32 && a->data_type != SML_INT32) return SML_ERR_UNSUPPORTED;
    if (a->count == 0) return SML_OK;
    if (!a->in && !a->out) return SML_ERR_INVALID_ARG;
    const uint64_t P = a->packet_numel;
    const uint64_t B = sml_num_blocks(a->numel, (uint32_t)P);
    const bool flt = a->data_type == SML_FLOAT32;
    const uint64_t b = flt || window ? a->batch_num_ltus : 0;
    if ((flt || window) && b > B) return SML_ERR_INVALID_ARG;
    if (window && b == 0) return SML_ERR_INVALID_ARG;
    if (flt && !a->recv_exps) return SML_ERR_INVALID_ARG;
    const uint64_t total = flt ? B + b : B;
    bool run = true;   // ids q0, q0 + 1, ... (a ring pass): distinct, and q0 + b is not among them if count <= b
    for (uint32_t i = 0; i < a->count; i++) {
        const uint64_t q = a->pkt_ids[i];
        if (q >= total || !a->entries[i] || (flt && q < B && !a->extras[i])) return SML_ERR_INVALID_ARG;
        if (window && flt && q + b < B && !a->extras[i]) return SML_ERR_INVALID_ARG;
        run = run && q == a->pkt_ids[0] + i;
    }
    if (run && (b == 0 || a->count <= b)) return SML_OK;
    // any other order: distinct, and never q and q + b together (sorted copy)
    uint64_t ids[SML_MAX_BURST];
    std::copy(a->pkt_ids, a->pkt_ids + a->count, ids);
    std::sort(ids, ids + a->count);
    for (uint32_t i = 1; i < a->count; i++)
        if (ids[i] == ids[i - 1]) return SML_ERR_INVALID_ARG;
    if (b)
        for (uint32_t i = 0; i < a->count; i++)
            if (std::binary_search(ids, ids + a->count, ids[i] + b)) return SML_ERR_INVALID_ARG;
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

sml_status_t sml_exchange_burst(const sml_packet_burst* burst, void* stream) {
    sml_status_t st = check_burst(burst, true);
    if (st != SML_OK || burst->count == 0) return st;
    if (!burst->in || !burst->out) return SML_ERR_INVALID_ARG;
    const sml_packet_burst& a = *burst;
    const dim3 grid((a.count + kWavesPerBlock - 1) / kWavesPerBlock);
    const hipStream_t s = (hipStream_t)stream;
    const bool rne = (a.flags & SML_FLAG_ROUND_RNE) != 0;
    const bool proc = (a.flags & SML_FLAG_PROCESS_PACKET) != 0;
#define SML_XCH(PN)                                                                                \
    if (proc) {                                                                                    \
        if (rne) k_exchange_burst<PN, true, true><<<grid, kBlockThreads, 0, s>>>(a);               \
        else k_exchange_burst<PN, false, true><<<grid, kBlockThreads, 0, s>>>(a);                  \
    } else {                                                                                       \
        if (rne) k_exchange_burst<PN, true, false><<<grid, kBlockThreads, 0, s>>>(a);              \
        else k_exchange_burst<PN, false, false><<<grid, kBlockThreads, 0, s>>>(a);                 \
    }
    switch (a.packet_numel) {
        case 64: SML_XCH(64) break;
        case 128: SML_XCH(128) break;
        case 256: SML_XCH(256) break;
        case 512: SML_XCH(512) break;
        default: SML_XCH(1024) break;
    }
#undef SML_XCH
    return launch_check();
}

}  // extern "C"

struct sml_burst_server {
    sml::ServerCtl* ctl = nullptr;    // host address (coherent, device-mapped)
    sml::ServerCtl* dctl = nullptr;   // the same memory at its device address
    uint32_t* arrive = nullptr;       // device memory: workgroups done with the current burst
    hipStream_t stream = nullptr;
    uint32_t packet_numel = 0;
    bool rne = false;
    uint64_t idle_ticks = 0;
    std::chrono::milliseconds restart_after{50};   // half the server's idle time
    uint64_t seq = 0;
    bool launched = false;            // a kernel was launched and not yet joined
    std::chrono::steady_clock::time_point last_activity;
};

namespace {

uint64_t host_load(const volatile uint64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

bool any_exited(const sml_burst_server* s) {
    for (int g = 0; g < sml::kServerGroups; g++)
        if (__atomic_load_n(&s->ctl->exited[g], __ATOMIC_ACQUIRE)) return true;
    return false;
}

// Stop a launched server (if any) and wait for every workgroup to leave.
sml_status_t server_join(sml_burst_server* s) {
    if (!s->launched) return SML_OK;
    __atomic_store_n(&s->ctl->stop, 1u, __ATOMIC_RELEASE);
    s->launched = false;
    return sml::hip_check(hipStreamSynchronize(s->stream));
}

sml_status_t server_launch(sml_burst_server* s) {
    sml_status_t st = server_join(s);
    if (st != SML_OK) return st;
    for (int g = 0; g < sml::kServerGroups; g++) __atomic_store_n(&s->ctl->exited[g], 0u, __ATOMIC_RELEASE);
    __atomic_store_n(&s->ctl->stop, 0u, __ATOMIC_RELEASE);
    // The new kernel starts from seen = done.  After a failed burst (timeout,
    // a workgroup's idle exit mid-burst) done lags the last doorbell; the
    // relaunched server would take that stale doorbell for a new burst and
    // replay its descriptor (an exchange burst applied twice, or buffers of a
    // finished slice).  No kernel runs here (joined above): mark every rung
    // doorbell as handled.
    __atomic_store_n(&s->ctl->done, s->seq, __ATOMIC_RELEASE);
    st = sml::hip_check(hipMemsetAsync(s->arrive, 0, sizeof(uint32_t), s->stream));
    if (st != SML_OK) return st;
    const dim3 grid(sml::kServerGroups), block(sml::kServerThreads);
#define SML_SRV(PN)                                                                                        \
    if (s->rne) sml::k_burst_server<PN, true><<<grid, block, 0, s->stream>>>(s->dctl, s->arrive, s->idle_ticks); \
    else sml::k_burst_server<PN, false><<<grid, block, 0, s->stream>>>(s->dctl, s->arrive, s->idle_ticks);
    switch (s->packet_numel) {
        case 64: SML_SRV(64) break;
        case 128: SML_SRV(128) break;
        case 256: SML_SRV(256) break;
        case 512: SML_SRV(512) break;
        default: SML_SRV(1024) break;
    }
#undef SML_SRV
    st = sml::launch_check();
    s->launched = st == SML_OK;
    s->last_activity = std::chrono::steady_clock::now();
    return st;
}

}  // namespace

extern "C" {

sml_status_t sml_burst_server_create(uint32_t packet_numel, uint32_t flags, uint32_t idle_ms,
                                     sml_burst_server** out) {
    if (!out) return SML_ERR_INVALID_ARG;
    *out = nullptr;
    if (!sml::valid_packet(packet_numel)) return SML_ERR_UNSUPPORTED;
    if (flags & ~SML_FLAG_ROUND_RNE) return SML_ERR_INVALID_ARG;
    int dev = 0, rate_khz = 0;
    sml_status_t st = sml::hip_check(hipGetDevice(&dev));
    if (st == SML_OK) st = sml::hip_check(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev));
    if (st != SML_OK) return st;
    auto* s = new sml_burst_server;
    const uint32_t ms = idle_ms ? idle_ms : 100;
    s->packet_numel = packet_numel;
    s->rne = (flags & SML_FLAG_ROUND_RNE) != 0;
    s->idle_ticks = (uint64_t)(rate_khz > 0 ? rate_khz : 100000) * ms;
    s->restart_after = std::chrono::milliseconds(ms / 2);
    void* h = nullptr;
    void* d = nullptr;
    st = sml::hip_check(hipHostMalloc(&h, sizeof(sml::ServerCtl), hipHostMallocMapped | hipHostMallocCoherent));
    if (st == SML_OK) {
        memset(h, 0, sizeof(sml::ServerCtl));
        st = sml::hip_check(hipHostGetDevicePointer(&d, h, 0));
    }
    if (st == SML_OK) st = sml::hip_check(hipMalloc(reinterpret_cast<void**>(&s->arrive), 64));
    if (st == SML_OK) st = sml::hip_check(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    if (st != SML_OK) {
        if (h) (void)hipHostFree(h);
        if (s->arrive) (void)hipFree(s->arrive);
        delete s;
        return st;
    }
    s->ctl = static_cast<sml::ServerCtl*>(h);
    s->dctl = static_cast<sml::ServerCtl*>(d);
    *out = s;
    return SML_OK;
}

sml_status_t sml_burst_server_submit(sml_burst_server* s, uint32_t op, const sml_packet_burst* burst) {
    if (!s || op > SML_BURST_EXCHANGE) return SML_ERR_INVALID_ARG;
    sml_status_t st = sml::check_burst(burst, op == SML_BURST_EXCHANGE);
    if (st != SML_OK || burst->count == 0) return st;
    if ((op != SML_BURST_POST && !burst->in) || (op != SML_BURST_PRE && !burst->out)) return SML_ERR_INVALID_ARG;
    if (burst->packet_numel != s->packet_numel || ((burst->flags & SML_FLAG_ROUND_RNE) != 0) != s->rne)
        return SML_ERR_INVALID_ARG;   // fixed per server
    // not running, left its loop, or close to its idle exit: (re)start it, so
    // the doorbell below never races an idle exit
    if (!s->launched || any_exited(s) ||
        std::chrono::steady_clock::now() - s->last_activity > s->restart_after) {
        st = server_launch(s);
        if (st != SML_OK) return st;
    }
    memcpy(&s->ctl->burst, burst, sizeof(sml_packet_burst));
    __atomic_store_n(&s->ctl->doorbell, (++s->seq << 2) | op, __ATOMIC_RELEASE);
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(10);
    for (uint32_t spins = 0; host_load(&s->ctl->done) != s->seq; spins++) {
        if ((spins & 255) != 255) continue;
        if (any_exited(s) && host_load(&s->ctl->done) != s->seq) {
            (void)server_join(s);
            strncpy(sml::g_last_error, "burst server: a workgroup left its loop during a burst",
                    sizeof(sml::g_last_error) - 1);
            return SML_ERR_HIP;
        }
        if (std::chrono::steady_clock::now() > t_end) {
            (void)server_join(s);
            strncpy(sml::g_last_error, "burst server: no completion within 10 s", sizeof(sml::g_last_error) - 1);
            return SML_ERR_HIP;
        }
    }
    s->last_activity = std::chrono::steady_clock::now();
    return SML_OK;
}

sml_status_t sml_burst_server_stop(sml_burst_server* s) {
    if (!s) return SML_ERR_INVALID_ARG;
    return server_join(s);
}

sml_status_t sml_burst_server_start(sml_burst_server* s) {
    if (!s) return SML_ERR_INVALID_ARG;
    if (s->launched && !any_exited(s)) return SML_OK;
    return server_launch(s);
}

sml_status_t sml_burst_server_inject_unanswered(sml_burst_server* s, uint32_t op, const sml_packet_burst* burst) {
    if (!s || !burst || op > SML_BURST_EXCHANGE) return SML_ERR_INVALID_ARG;
    const sml_status_t st = server_join(s);
    if (st != SML_OK) return st;
    memcpy(&s->ctl->burst, burst, sizeof(sml_packet_burst));
    __atomic_store_n(&s->ctl->doorbell, (++s->seq << 2) | op, __ATOMIC_RELEASE);
    return SML_OK;
}

sml_status_t sml_burst_server_destroy(sml_burst_server* s) {
    if (!s) return SML_OK;
    const sml_status_t st = sml_burst_server_stop(s);
    (void)hipStreamDestroy(s->stream);
    (void)hipFree(s->arrive);
    (void)hipHostFree(s->ctl);
    delete s;
    return st;
}

}  // extern "C"
