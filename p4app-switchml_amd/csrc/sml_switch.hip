// sml_switch.hip — the switch's aggregation over W worker planes as a CDNA4
// kernel (K6), with the worker's dequantize fused behind it.
//
// The Tofino data plane adds the W workers' payload slots as bit<32>
// (p4/processor.p4:48-54, wrapping) after parsing them big-endian, takes the
// signed int8 max of the exponents (p4/exponents.p4:48-54, types.p4:113,119)
// and multicasts the result; every worker then runs PostprocessSingle
// (ppp.cc:197-251) with scale(W, e_max).  Here the W planes are device
// pointers — local buffers, or peers' HBM mapped over xGMI (IPC handles) — so
// one pass reads W payload planes and writes the aggregated plane and/or the
// dequantized fp32 bucket:
//   payload_out[i] = htonl(sum_w ntohl(payload_w[i]))   (LE words: no swaps)
//   exps_out[k]    = max_w (int8) exps_w[k]
//   out[i]         = (float)(int32)sum_i / scale(W, e_max[i / P])
// Bit-identical to orc_switch_payload / orc_switch_exps followed by K4.
#include "sml_host.h"

namespace sml {

// The reader's half of a hand-off from other GPUs (SML_FLAG_PEER_PLANES):
// one system-scope acquire per workgroup before any load — on gfx950
// `buffer_inv sc0 sc1`, which invalidates this CU's L1 and the XCD L2's
// non-local lines (peer HBM is cached as such) — then the wait that holds
// the workgroup until the invalidate is done (MI355X_MICROARCH.md: the
// consumer's acquire -> s_waitcnt vmcnt(0) -> barrier -> plain loads).
__device__ __forceinline__ void acquire_peer_planes(uint32_t flags) {
    if (flags & SML_FLAG_PEER_PLANES) {   // uniform over the launch
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
}

// The writer's half (sml_release_to_peers): a system-scope release from
// kReleaseBlocks workgroups.  Workgroups are dealt round-robin over the 8
// XCDs, so every XCD's L2 is written back by several of them (one per XCD
// would do; the surplus costs nothing measurable and does not depend on the
// dispatcher's exact placement).
constexpr uint32_t kReleaseBlocks = 256;

__global__ __launch_bounds__(64) void k_release_to_peers() {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

struct SwitchArgs {
    const u4* payload[SML_MAX_SWITCH_WORKERS];
    const int8_t* exps[SML_MAX_SWITCH_WORKERS];
    u4* payload_out;        // nullable: aggregated plane (B*P words)
    int8_t* exps_out;       // nullable: max exponents (B bytes)
    float* out;             // nullable: dequantized bucket (numel floats)
    uint64_t numel;
    uint64_t nblocks;       // B
    uint64_t ntiles;        // ceil(B*P / 1024)
    uint32_t nw;            // planes = num_workers
    uint32_t xcd;
    uint32_t exps_scalar;   // every exps[w] 4-byte aligned: one scalar load per slice
    uint32_t flags;         // SML_FLAG_PEER_PLANES: acquire first
};

// W payload loads per lane-slice are issued before the adds (16-B
// non-temporal, as K4); exponent bytes come one scalar load per slice and
// plane when the planes are 4-byte aligned.
template <int P, bool ALIGNED, bool BE, bool RCP, bool EXPS>
__global__ __launch_bounds__(kBlockThreads) void k_switch_aggregate(SwitchArgs a) {
    __shared__ float lut[256];
    acquire_peer_planes(a.flags);
    if (a.out) {
        if constexpr (RCP) build_rcp_lut(lut, a.nw);
        else build_lut(lut, a.nw);
    }
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t padded = a.nblocks * P;
    for (uint64_t t = xcd_block(a.xcd) * kWavesPerBlock + wave_index(); t < a.ntiles; t += nwaves) {
        const uint64_t base = t * kTileElems;
        const bool full = base + kTileElems <= padded;
        u4 acc[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) acc[u] = mku4(0, 0, 0, 0);
#pragma unroll 2   // two planes' loads issued together per trip (profiles/r01/ab11_switch_unroll.json)
        for (uint32_t w = 0; w < a.nw; w++) {
            u4 v[kU];
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4;
                v[u] = (full || idx < padded) ? __builtin_nontemporal_load(a.payload[w] + idx / 4) : mku4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < kU; u++) {
                if constexpr (BE) {
                    acc[u].x += bswap(v[u].x); acc[u].y += bswap(v[u].y);
                    acc[u].z += bswap(v[u].z); acc[u].w += bswap(v[u].w);
                } else {
                    acc[u].x += v[u].x; acc[u].y += v[u].y; acc[u].z += v[u].z; acc[u].w += v[u].w;
                }
            }
        }
        int e[kU];
        if constexpr (EXPS) {
#pragma unroll
            for (int u = 0; u < kU; u++) e[u] = -128;
            for (uint32_t w = 0; w < a.nw; w++) {
                if (full && a.exps_scalar) {
#pragma unroll
                    for (int u = 0; u < kU; u++) {
                        const int ew = (int)(int8_t)(uint8_t)slice_exponent_byte<P>(a.exps[w], base, u, lane);
                        e[u] = ew > e[u] ? ew : e[u];
                    }
                } else {
#pragma unroll
                    for (int u = 0; u < kU; u++) {
                        const uint64_t pkt = (base + (uint64_t)(u * kWave + lane) * 4) / P;
                        const int ew = pkt < a.nblocks ? (int)a.exps[w][pkt] : -128;
                        e[u] = ew > e[u] ? ew : e[u];
                    }
                }
            }
            if (a.exps_out) {
                constexpr int kPk = kTileElems / P;
                if (((uintptr_t)a.exps_out & (kPk - 1)) == 0 && full)
                    store_tile_exponents<P>(a.exps_out + base / P, lane, e);
                else
                    store_exponents<P>(a.exps_out, base, lane, e, a.nblocks);
            }
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4;
            if (!full && idx >= padded) continue;
            if (a.payload_out) {
                const u4 q = acc[u];
                store_payload(a.payload_out + idx / 4,
                              BE ? mku4(bswap(q.x), bswap(q.y), bswap(q.z), bswap(q.w)) : q);
            }
            if constexpr (EXPS) {
                if (a.out && idx < a.numel) {
                    const float s = lut[(uint8_t)e[u]];
                    const u4 q = acc[u];
                    f4 o;
                    if constexpr (RCP)
                        o = mkf4((float)(int32_t)q.x * s, (float)(int32_t)q.y * s, (float)(int32_t)q.z * s,
                                 (float)(int32_t)q.w * s);
                    else
                        o = mkf4(dequantize1(q.x, s), dequantize1(q.y, s), dequantize1(q.z, s), dequantize1(q.w, s));
                    if (idx + 4 <= a.numel) store4<ALIGNED>(a.out + idx, o);
                    else store4_guarded(a.out + idx, o, idx, a.numel);
                }
            }
        }
    }
}

// Exponent max over W planes, 4 blocks per thread (one dword per plane when
// every plane is 4-byte aligned, bytes otherwise).
struct ExpsMaxArgs {
    const int8_t* exps[SML_MAX_SWITCH_WORKERS];
    int8_t* out;
    uint64_t nblocks;
    uint32_t nw;
    uint32_t aligned;
    uint32_t flags;
};

__global__ __launch_bounds__(kBlockThreads) void k_switch_exps(ExpsMaxArgs a) {
    acquire_peer_planes(a.flags);
    const uint64_t stride = (uint64_t)gridDim.x * kBlockThreads;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlockThreads + threadIdx.x; 4 * i < a.nblocks; i += stride) {
        const uint64_t k0 = 4 * i;
        if (a.aligned && k0 + 4 <= a.nblocks) {
            int m0 = -128, m1 = -128, m2 = -128, m3 = -128;
            for (uint32_t w = 0; w < a.nw; w++) {
                const uint32_t d = *reinterpret_cast<const uint32_t*>(a.exps[w] + k0);
                const int e0 = (int8_t)(d & 0xff), e1 = (int8_t)((d >> 8) & 0xff);
                const int e2 = (int8_t)((d >> 16) & 0xff), e3 = (int8_t)(d >> 24);
                m0 = e0 > m0 ? e0 : m0; m1 = e1 > m1 ? e1 : m1; m2 = e2 > m2 ? e2 : m2; m3 = e3 > m3 ? e3 : m3;
            }
            *reinterpret_cast<uint32_t*>(a.out + k0) =
                (uint32_t)(uint8_t)m0 | ((uint32_t)(uint8_t)m1 << 8) | ((uint32_t)(uint8_t)m2 << 16) |
                ((uint32_t)(uint8_t)m3 << 24);
        } else {
            for (uint64_t k = k0; k < k0 + 4 && k < a.nblocks; k++) {
                int m = -128;
                for (uint32_t w = 0; w < a.nw; w++) m = a.exps[w][k] > m ? a.exps[w][k] : m;
                a.out[k] = (int8_t)m;
            }
        }
    }
}

struct CopyOp {
    __device__ __forceinline__ uint32_t operator()(uint32_t q) const { return q; }
};

// The in-node switch's multicast: the W workers' shards gathered in ONE
// launch.  Copied one after another, each shard would come over one peer's
// xGMI link at a time; here the tiles are dealt round-robin over the
// segments in groups of kSegGroup (64 KiB of words), so every resident wave
// set reads from all W peers — all links at once — while each group stays a
// contiguous run.  Group g of the launch: segment g % nseg, that segment's
// group g / nseg (idle once the segment is done: shards differ by at most one
// block's words).
constexpr uint32_t kSegGroup = 16;   // tiles per group

struct SegCopyArgs {
    const uint32_t* src[SML_MAX_SWITCH_WORKERS];
    uint32_t* dst[SML_MAX_SWITCH_WORKERS];
    uint64_t n[SML_MAX_SWITCH_WORKERS];
    uint32_t nseg;
    uint64_t ntiles;        // nseg x (the largest segment's groups) x kSegGroup
    uint32_t xcd;
    uint32_t flags;
};

__global__ __launch_bounds__(kBlockThreads) void k_copy_segments(SegCopyArgs a) {
    acquire_peer_planes(a.flags);
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t t = xcd_block(a.xcd) * kWavesPerBlock + wave_index(); t < a.ntiles; t += nwaves) {
        const uint64_t g = t / kSegGroup;
        const uint32_t s = (uint32_t)(g % a.nseg);
        const uint64_t base = ((g / a.nseg) * kSegGroup + t % kSegGroup) * (uint64_t)kTileElems;
        const uint64_t n = a.n[s];
        if (base >= n) continue;
        const uint32_t* in = a.src[s];
        uint32_t* out = a.dst[s];
        if (base + kTileElems <= n) {
            u4a v[kU];
#pragma unroll
            for (int u = 0; u < kU; u++)
                v[u] = __builtin_nontemporal_load(reinterpret_cast<const u4a*>(in + base + (u * kWave + lane) * 4));
#pragma unroll
            for (int u = 0; u < kU; u++) *reinterpret_cast<u4a*>(out + base + (u * kWave + lane) * 4) = v[u];
        } else {
#pragma unroll
            for (int u = 0; u < kU; u++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4 + j;
                    if (idx < n) out[idx] = in[idx];
                }
        }
    }
}

template <bool ALIGNED, bool BE, bool RCP, bool EXPS>
static void launch_switch_p(uint32_t P, dim3 grid, hipStream_t st, const SwitchArgs& a) {
    switch (P) {
        case 64:   k_switch_aggregate<64, ALIGNED, BE, RCP, EXPS><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 128:  k_switch_aggregate<128, ALIGNED, BE, RCP, EXPS><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 256:  k_switch_aggregate<256, ALIGNED, BE, RCP, EXPS><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 512:  k_switch_aggregate<512, ALIGNED, BE, RCP, EXPS><<<grid, kBlockThreads, 0, st>>>(a); break;
        default:   k_switch_aggregate<1024, ALIGNED, BE, RCP, EXPS><<<grid, kBlockThreads, 0, st>>>(a); break;
    }
}

template <bool ALIGNED, bool BE>
static void launch_switch_m(bool exps, bool rcp, uint32_t P, dim3 g, hipStream_t st, const SwitchArgs& a) {
    if (!exps) launch_switch_p<ALIGNED, BE, false, false>(P, g, st, a);
    else if (rcp) launch_switch_p<ALIGNED, BE, true, true>(P, g, st, a);
    else launch_switch_p<ALIGNED, BE, false, true>(P, g, st, a);
}

// ncclUint8 buckets (the CollNet plugin, switchml_plugin.cc:318-337 and
// 370-378): widened to int32 for the INT32 all-reduce, narrowed back (mod 256).
__global__ __launch_bounds__(kBlockThreads) void k_widen_u8(const uint8_t* in, int32_t* out, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlockThreads;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlockThreads + threadIdx.x; i < n; i += stride) out[i] = in[i];
}

__global__ __launch_bounds__(kBlockThreads) void k_narrow_u8(const int32_t* in, uint8_t* out, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlockThreads;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlockThreads + threadIdx.x; i < n; i += stride)
        out[i] = (uint8_t)in[i];
}

}  // namespace sml

using namespace sml;

extern "C" {

sml_status_t sml_switch_aggregate(const int32_t* const* d_payloads, const int8_t* const* d_exps,
                                  uint16_t num_workers, uint64_t numel, uint32_t packet_numel,
                                  int32_t* d_payload_out, int8_t* d_exps_out, float* d_out,
                                  uint32_t flags, void* stream) {
    if (!valid_packet(packet_numel)) return SML_ERR_UNSUPPORTED;
    if (num_workers == 0 || !d_payloads) return SML_ERR_INVALID_ARG;
    if (num_workers > SML_MAX_SWITCH_WORKERS) return SML_ERR_UNSUPPORTED;
    if (numel == 0) return SML_OK;
    if (!d_payload_out && !d_exps_out && !d_out) return SML_ERR_INVALID_ARG;
    const bool exps = d_exps_out || d_out;
    if (exps && !d_exps) return SML_ERR_INVALID_ARG;
    if (d_out && !aligned4(d_out)) return SML_ERR_INVALID_ARG;
    if (d_payload_out && !aligned16(d_payload_out)) return SML_ERR_ALIGNMENT;
    SwitchArgs a{};
    a.exps_scalar = 1;
    for (uint32_t w = 0; w < num_workers; w++) {
        if (!d_payloads[w]) return SML_ERR_INVALID_ARG;
        if (!aligned16(d_payloads[w])) return SML_ERR_ALIGNMENT;
        a.payload[w] = reinterpret_cast<const u4*>(d_payloads[w]);
        if (exps) {
            if (!d_exps[w]) return SML_ERR_INVALID_ARG;
            a.exps[w] = d_exps[w];
            if (!aligned4(d_exps[w])) a.exps_scalar = 0;
        }
    }
    a.payload_out = reinterpret_cast<u4*>(d_payload_out);
    a.exps_out = d_exps_out;
    a.out = d_out;
    a.numel = numel;
    a.nblocks = sml_num_blocks(numel, packet_numel);
    a.ntiles = (a.nblocks * packet_numel + kTileElems - 1) / kTileElems;
    a.nw = num_workers;
    a.xcd = g_xcd_chunk.load(std::memory_order_relaxed);
    a.flags = flags & SML_FLAG_PEER_PLANES;
    const dim3 grid(grid_for_tiles(a.ntiles));
    const hipStream_t st = (hipStream_t)stream;
    const bool al = !d_out || aligned16(d_out), be = !(flags & SML_FLAG_PAYLOAD_LE);
    const bool rcp = (num_workers & (num_workers - 1)) == 0;
    if (al) { if (be) launch_switch_m<true, true>(exps, rcp, packet_numel, grid, st, a);
              else launch_switch_m<true, false>(exps, rcp, packet_numel, grid, st, a); }
    else    { if (be) launch_switch_m<false, true>(exps, rcp, packet_numel, grid, st, a);
              else launch_switch_m<false, false>(exps, rcp, packet_numel, grid, st, a); }
    return launch_check();
}

sml_status_t sml_switch_exps(const int8_t* const* d_exps, uint16_t num_workers, uint64_t num_blocks,
                             int8_t* d_exps_out, uint32_t flags, void* stream) {
    if (num_workers == 0 || !d_exps || !d_exps_out) return SML_ERR_INVALID_ARG;
    if (num_workers > SML_MAX_SWITCH_WORKERS) return SML_ERR_UNSUPPORTED;
    if (num_blocks == 0) return SML_OK;
    ExpsMaxArgs a{};
    a.aligned = aligned4(d_exps_out);
    for (uint32_t w = 0; w < num_workers; w++) {
        if (!d_exps[w]) return SML_ERR_INVALID_ARG;
        a.exps[w] = d_exps[w];
        if (!aligned4(d_exps[w])) a.aligned = 0;
    }
    a.out = d_exps_out;
    a.nblocks = num_blocks;
    a.nw = num_workers;
    a.flags = flags & SML_FLAG_PEER_PLANES;
    k_switch_exps<<<grid_for_vec((num_blocks + 3) / 4), kBlockThreads, 0, (hipStream_t)stream>>>(a);
    return launch_check();
}

sml_status_t sml_copy_words(const void* d_src, void* d_dst, uint64_t num_words, void* stream) {
    if (num_words == 0) return SML_OK;
    if (!d_src || !d_dst || !aligned4(d_src) || !aligned4(d_dst)) return SML_ERR_INVALID_ARG;
    const uint64_t ntiles = (num_words + kTileElems - 1) / kTileElems;
    k_words<<<grid_for_tiles(ntiles), kBlockThreads, 0, (hipStream_t)stream>>>(
        static_cast<const uint32_t*>(d_src), static_cast<uint32_t*>(d_dst), num_words,
        g_xcd_chunk.load(std::memory_order_relaxed), CopyOp{});
    return launch_check();
}

// ncclUint8 buckets of the CollNet plugin (kernels above).
sml_status_t sml_widen_u8_i32(const uint8_t* d_in, int32_t* d_out, uint64_t n, void* stream) {
    if (n == 0) return SML_OK;
    if (!d_in || !d_out || !aligned4(d_out)) return SML_ERR_INVALID_ARG;
    k_widen_u8<<<grid_for_vec(n), kBlockThreads, 0, (hipStream_t)stream>>>(d_in, d_out, n);
    return launch_check();
}

sml_status_t sml_narrow_i32_u8(const int32_t* d_in, uint8_t* d_out, uint64_t n, void* stream) {
    if (n == 0) return SML_OK;
    if (!d_in || !d_out || !aligned4(d_in)) return SML_ERR_INVALID_ARG;
    k_narrow_u8<<<grid_for_vec(n), kBlockThreads, 0, (hipStream_t)stream>>>(d_in, d_out, n);
    return launch_check();
}

sml_status_t sml_copy_segments(const void* const* d_srcs, void* const* d_dsts, const uint64_t* num_words,
                               uint32_t num_segments, uint32_t flags, void* stream) {
    if (num_segments == 0) return SML_OK;
    if (!d_srcs || !d_dsts || !num_words || num_segments > SML_MAX_SWITCH_WORKERS) return SML_ERR_INVALID_ARG;
    SegCopyArgs a;
    a.nseg = 0;
    uint64_t groups = 0;
    const uint64_t gw = (uint64_t)kSegGroup * kTileElems;   // words per group
    for (uint32_t i = 0; i < num_segments; i++) {
        if (num_words[i] == 0) continue;                    // empty segments touch nothing
        if (!d_srcs[i] || !d_dsts[i] || !aligned4(d_srcs[i]) || !aligned4(d_dsts[i])) return SML_ERR_INVALID_ARG;
        a.src[a.nseg] = static_cast<const uint32_t*>(d_srcs[i]);
        a.dst[a.nseg] = static_cast<uint32_t*>(d_dsts[i]);
        a.n[a.nseg] = num_words[i];
        const uint64_t gi = (num_words[i] + gw - 1) / gw;
        groups = gi > groups ? gi : groups;
        a.nseg++;
    }
    if (a.nseg == 0) return SML_OK;
    a.ntiles = (uint64_t)a.nseg * groups * kSegGroup;
    a.xcd = g_xcd_chunk.load(std::memory_order_relaxed);
    a.flags = flags & SML_FLAG_PEER_PLANES;
    k_copy_segments<<<grid_for_tiles(a.ntiles), kBlockThreads, 0, (hipStream_t)stream>>>(a);
    return launch_check();
}

sml_status_t sml_release_to_peers(void* stream) {
    k_release_to_peers<<<kReleaseBlocks, 64, 0, (hipStream_t)stream>>>();
    return launch_check();
}

}  // extern "C"

// ---- plane sharing for the peer-to-peer switch (hipIpc*) ----------------
extern "C" {

uint32_t sml_ipc_handle_bytes(void) { return (uint32_t)sizeof(hipIpcMemHandle_t); }

sml_status_t sml_ipc_get_handle(const void* d_ptr, void* handle_out, uint64_t* offset_out) {
    if (!d_ptr || !handle_out || !offset_out) return SML_ERR_INVALID_ARG;
    // the handle names the whole allocation (a caching allocator may have
    // sub-allocated d_ptr from it): report where d_ptr lies inside it
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    sml_status_t s = hip_check(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)d_ptr));
    if (s != SML_OK) return s;
    hipIpcMemHandle_t h;
    s = hip_check(hipIpcGetMemHandle(&h, (void*)base));
    if (s != SML_OK) return s;
    memcpy(handle_out, &h, sizeof(h));
    *offset_out = (uint64_t)((const char*)d_ptr - (const char*)base);
    return SML_OK;
}

sml_status_t sml_ipc_open_handle(const void* handle, void** d_ptr_out) {
    if (!handle || !d_ptr_out) return SML_ERR_INVALID_ARG;
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    return hip_check(hipIpcOpenMemHandle(d_ptr_out, h, hipIpcMemLazyEnablePeerAccess));
}

sml_status_t sml_ipc_close_handle(void* d_ptr) {
    if (!d_ptr) return SML_ERR_INVALID_ARG;
    return hip_check(hipIpcCloseMemHandle(d_ptr));
}

}  // extern "C"
