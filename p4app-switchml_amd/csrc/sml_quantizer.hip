// sml_quantizer.hip — CDNA4 (gfx950) kernels for the planes of SwitchML's
// end-host pre/post-processor (CpuExponentQuantizerPPP,
// client_lib/src/prepostprocessors/cpu_exponent_quantizer_ppp.cc = "ppp.cc")
// and their C-ABI entry points (include/switchml_hip.h): K1 fused exponent +
// quantize + pack, K2 exponents, K3 quantize with given exponents, K4
// dequantize, the fused loopback round trip, the word streams (loopback x W,
// INT32 byteswap), RDMA immediates and the copy probe.  Tile layout, numerics
// and parity notes: sml_device.h; DPDK frames: sml_frames.hip.
#include "sml_host.h"


namespace sml {

thread_local char g_last_error[256] = "";
std::atomic<uint32_t> g_grid_limit{0};
std::atomic<uint32_t> g_xcd_chunk{64};

// -------------------------------------------------------------- kernels

// K3: the tile's global exponents (one scalar load per slice when aligned).
template <int P, int U>
__device__ __forceinline__ void global_tile_exponents(const QuantArgs& a, uint64_t base, int lane, int (&e)[U]) {
    if (base + tile_elems<U>() <= a.nblocks * P && slice_exps_scalar_ok<P>(a.gexp)) {
#pragma unroll
        for (int u = 0; u < U; u++) e[u] = (int)(int8_t)slice_exponent_byte<P>(a.gexp, base, u, lane);
    } else {
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint64_t pkt = (base + (uint64_t)(u * kWave + lane) * 4) / P;
            e[u] = pkt < a.nblocks ? (int)a.gexp[pkt] : 0;
        }
    }
}

// Quantize + pack 4 consecutive elements (one lane's part of a slice).
template <int P, bool BE, bool RNE, bool NTS>
__device__ __forceinline__ void quant_slice(const QuantArgs& a, uint64_t idx, f4 v, const float* lut, int e) {
    const float s = lut[(uint8_t)e];
    uint64_t body = 0;
    if constexpr (RNE) {
        // VCL body = first n - n%16 elements of the block; only the last
        // (partial) block has a scalar half-away tail.
        const uint64_t blk0 = idx / P * P;
        const uint64_t n = a.numel - blk0 < (uint64_t)P ? a.numel - blk0 : (uint64_t)P;
        body = blk0 + (n - n % 16);
    }
    u4 q = quantize4<RNE>(v, s, idx, body);
    if constexpr (BE) { q.x = bswap(q.x); q.y = bswap(q.y); q.z = bswap(q.z); q.w = bswap(q.w); }
    store_payload_as<NTS>(a.payload + idx / 4, q);
}

// Exponents, quantize and pack of one loaded tile (K3: `e` holds the global
// exponents already).
template <int P, bool GLOBAL, bool BE, bool RNE, int U, bool NTS>
__device__ __forceinline__ void quant_tile(const QuantArgs& a, uint64_t base, int lane, const f4 (&v)[U],
                                           const float* lut, int (&e)[U]) {
    const uint64_t padded = a.nblocks * P;
    constexpr int kElems = tile_elems<U>();
    if constexpr (!GLOBAL) {
        tile_exponents<P>(v, e);
        if (a.exps_out) {
            constexpr int kPk = kElems / P;       // packets per tile
            if (((uintptr_t)a.exps_out & (kPk - 1)) == 0 && base + kElems <= padded) {
                store_tile_exponents<P>(a.exps_out + base / P, lane, e);
            } else {
                store_exponents<P>(a.exps_out, base, lane, e, a.nblocks);
            }
        }
    }
    if (!a.payload) return;
    // A tile inside the padded plane takes a branch-free slice loop.  With a
    // per-slice `continue` here, hipcc's wait-count pass sees paths that skip
    // a slice and waits vmcnt(0) at the top of EVERY slice — i.e. on the
    // previous slice's store as well — which cost K3 (whose first use of the
    // loaded data is inside this loop) 3 % against K1 (whose exponent reduce
    // consumes all four slices first): profiles/r02/k1_vs_k3_counters.json,
    // ab_k3_waitcnt.json.
    if (base + kElems <= padded) {
#pragma unroll
        for (int u = 0; u < U; u++) quant_slice<P, BE, RNE, NTS>(a, base + (uint64_t)(u * kWave + lane) * 4, v[u], lut, e[u]);
        return;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4;
        if (idx < padded) quant_slice<P, BE, RNE, NTS>(a, idx, v[u], lut, e[u]);
    }
}

// K1 (fused exponent + quantize + pack), K2 (exponents only: payload == nullptr)
// and K3 (given global exponents: GLOBAL = true).  A wave's tile is U slices
// of 256 elements (one 16-B load per lane per slice, all issued before any
// arithmetic); U = 4 by default — four loads in flight per lane keep the
// stream at the copy rate, smaller tiles measured slower.
template <int P, bool ALIGNED, bool GLOBAL, bool BE, bool RNE, int U, bool NTS = false>
__global__ __launch_bounds__(kBlockThreads) void k_quantize_pack(QuantArgs a) {
    __shared__ float lut[256];
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    // The wave's first tile is loaded BEFORE the workgroup builds its scale
    // table: the table and its barrier run while the loads are in flight (a
    // plain s_barrier does not wait for them), instead of delaying the first
    // HBM request of every workgroup of the one-shot grid: K1 +1.1 / +1.7 %
    // at 256 / 128 MiB (profiles/r04/ab_lut_early.json).
    uint64_t t = xcd_block(a.xcd) * kWavesPerBlock + wave_index();
    f4 v[U];
    if (t < a.ntiles) load_tile<ALIGNED>(a, t * tile_elems<U>(), lane, v);
    if (a.payload) build_lut(lut, a.W);
    while (t < a.ntiles) {
        const uint64_t base = t * tile_elems<U>();
        int e[U];
        // K3: the exponent dword is read after the data loads are in flight
        if constexpr (GLOBAL) global_tile_exponents<P>(a, base, lane, e);
        quant_tile<P, GLOBAL, BE, RNE, U, NTS>(a, base, lane, v, lut, e);
        t += nwaves;
        if (t < a.ntiles) load_tile<ALIGNED>(a, t * tile_elems<U>(), lane, v);
    }
}

// ntohl (BE) -> int -> float, divided by the scale (or multiplied by its
// exact reciprocal, RCP) — PostprocessSingle's per-element arithmetic.
template <bool BE, bool RCP>
__device__ __forceinline__ f4 dequant_words(u4 w, float s) {
    uint32_t q0 = (uint32_t)w.x, q1 = (uint32_t)w.y, q2 = (uint32_t)w.z, q3 = (uint32_t)w.w;
    if constexpr (BE) { q0 = bswap(q0); q1 = bswap(q1); q2 = bswap(q2); q3 = bswap(q3); }
    if constexpr (RCP)
        return mkf4((float)(int32_t)q0 * s, (float)(int32_t)q1 * s, (float)(int32_t)q2 * s, (float)(int32_t)q3 * s);
    else
        return mkf4(dequantize1(q0, s), dequantize1(q1, s), dequantize1(q2, s), dequantize1(q3, s));
}

struct DequantArgs {
    const u4* payload;
    const int8_t* exps;
    float* out;
    uint64_t numel;
    uint64_t ntiles;        // ceil(numel / 1024)
    uint32_t W;
    uint32_t xcd;           // xcd_block chunk (0 = plain order)
};

// K4: dequantize the aggregated payload (PostprocessSingle, ppp.cc:197-251).
// RCP (power-of-two W): multiply by the exact reciprocal instead of the IEEE
// division — same bits (rcp_scale_pow2).
template <int P, bool ALIGNED, bool BE, bool RCP, bool NT = false, int U = kU>
__global__ __launch_bounds__(kBlockThreads) void k_dequantize(DequantArgs a) {
    __shared__ float lut[256];
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    constexpr int kElems = tile_elems<U>();
    uint64_t t = xcd_block(a.xcd) * kWavesPerBlock + wave_index();
    if constexpr (RCP) build_rcp_lut(lut, a.W);
    else build_lut(lut, a.W);
    for (; t < a.ntiles; t += nwaves) {
        const uint64_t base = t * kElems;
        const bool full = base + kElems <= a.numel;
        u4 w[U];
        float s[U];
        if (full && slice_exps_scalar_ok<P>(a.exps)) {
            // Full tile: each slice's exponent bytes with one scalar load
            // (measured: a per-lane byte load per slice costs ~8 % at
            // P != 256), then a branch-free slice loop — shared per-slice
            // blocks with the partial-tile path made hipcc wait vmcnt(0), on
            // the previous slice's store too, before every slice.
#pragma unroll
            for (int u = 0; u < U; u++) {
                w[u] = __builtin_nontemporal_load(a.payload + (base + (uint64_t)(u * kWave + lane) * 4) / 4);
                s[u] = lut[slice_exponent_byte<P>(a.exps, base, u, lane)];
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4;
                store4<ALIGNED, NT>(a.out + idx, dequant_words<BE, RCP>(w[u], s[u]));
            }
            continue;
        } else {
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4;
                if (full || idx < a.numel) {
                    w[u] = __builtin_nontemporal_load(a.payload + idx / 4);
                    s[u] = lut[(uint8_t)a.exps[idx / P]];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4;
            if (!full && idx >= a.numel) continue;
            const f4 o = dequant_words<BE, RCP>(w[u], s[u]);
            if (full) store4<ALIGNED, NT>(a.out + idx, o);
            else store4_guarded(a.out + idx, o, idx, a.numel);
        }
    }
}

struct RoundTripArgs {
    const float* in;
    float* out;
    uint64_t numel;
    uint64_t nblocks;
    uint64_t ntiles;        // ceil(B*P / 1024)
    u4* payload;          // nullable: on-wire plane as sent
    int8_t* exps_out;       // nullable
    uint32_t W;
    uint32_t xcd;           // xcd_block chunk (0 = plain order)
};

// Fused dummy-backend round trip: PreprocessSingle -> ProcessPacket (x W) ->
// PostprocessSingle for every packet of the slice in one HBM pass.  One tile
// of one slice (blocks restart at the slice start, as in the reference):
// roundtrip_load issues the tile's loads, roundtrip_compute does the rest.
template <bool ALIGNED, int U>
__device__ __forceinline__ void roundtrip_load(const RoundTripArgs& a, uint64_t t, int lane, f4 (&v)[U]) {
    constexpr int kElems = tile_elems<U>();
    const uint64_t base = t * kElems;
    if (base + kElems <= a.numel) {
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = load4<ALIGNED>(a.in + base + (u * kWave + lane) * 4);
    } else {
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4;
            v[u] = load4_guarded(a.in + idx, idx, a.numel);
        }
    }
}

template <int P, bool ALIGNED, bool BE, bool RNE, bool NT, int U>
__device__ __forceinline__ void roundtrip_compute(const RoundTripArgs& a, uint64_t t, const float* lut, int lane,
                                                  const f4 (&v)[U]) {
    static_assert(U * 256 >= P, "a tile holds whole packets");
    constexpr int kElems = tile_elems<U>();
    const bool pow2 = (a.W & (a.W - 1)) == 0;
    const uint32_t log2W = 31 - __builtin_clz(a.W);
    const uint64_t padded = a.nblocks * P;
    const uint64_t base = t * kElems;
    const bool full = base + kElems <= a.numel;
    int e[U];
    tile_exponents<P>(v, e);
    if (a.exps_out) {
        constexpr int kPk = kElems / P;
        if (((uintptr_t)a.exps_out & (kPk - 1)) == 0 && base + kElems <= padded)
            store_tile_exponents<P>(a.exps_out + base / P, lane, e);
        else
            store_exponents<P>(a.exps_out, base, lane, e, a.nblocks);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4;
        if (idx >= padded) continue;
        const float s = lut[(uint8_t)e[u]];
        uint64_t body = 0;
        if constexpr (RNE) {
            const uint64_t blk0 = idx / P * P;
            const uint64_t n = a.numel - blk0 < (uint64_t)P ? a.numel - blk0 : (uint64_t)P;
            body = blk0 + (n - n % 16);
        }
        const u4 qv = quantize4<RNE>(v[u], s, idx, body);
        const uint32_t q[4] = {qv.x, qv.y, qv.z, qv.w};
        if (a.payload) {
            u4 wq = BE ? mku4(bswap(q[0]), bswap(q[1]), bswap(q[2]), bswap(q[3]))
                          : mku4(q[0], q[1], q[2], q[3]);
            store_payload(a.payload + idx / 4, wq);
        }
        // DummyBackend::ProcessPacket: int32 wrap multiply by W; then the
        // dequantize (exact reciprocal multiply for power-of-two W, as K4).
        f4 o;
        if (pow2) {
            const float r = rcp_scale_pow2(log2W, e[u]);
            o = mkf4((float)(int32_t)(q[0] * a.W) * r, (float)(int32_t)(q[1] * a.W) * r,
                     (float)(int32_t)(q[2] * a.W) * r, (float)(int32_t)(q[3] * a.W) * r);
        } else {
            o = mkf4(dequantize1(q[0] * a.W, s), dequantize1(q[1] * a.W, s), dequantize1(q[2] * a.W, s),
                     dequantize1(q[3] * a.W, s));
        }
        if (full) store4<ALIGNED, NT>(a.out + idx, o);
        else if (idx < a.numel) store4_guarded(a.out + idx, o, idx, a.numel);
    }
}

template <int P, bool ALIGNED, bool BE, bool RNE, bool NT = false, int U = kU>
__device__ __forceinline__ void roundtrip_tile(const RoundTripArgs& a, uint64_t t, const float* lut, int lane) {
    f4 v[U];
    roundtrip_load<ALIGNED, U>(a, t, lane, v);
    roundtrip_compute<P, ALIGNED, BE, RNE, NT, U>(a, t, lut, lane, v);
}

template <int P, bool ALIGNED, bool BE, bool RNE, bool NT = false, int U = kU>
__global__ __launch_bounds__(kBlockThreads) void k_roundtrip(RoundTripArgs a) {
    __shared__ float lut[256];
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    uint64_t t = xcd_block(a.xcd) * kWavesPerBlock + wave_index();
    // As K1: the first tile's loads go out before the scale table is built
    // (measured level here, +0.1-0.3 %: profiles/r04/ab_lut_early2.json).
    f4 v[U];
    if (t < a.ntiles) roundtrip_load<ALIGNED, U>(a, t, lane, v);
    build_lut(lut, a.W);
    while (t < a.ntiles) {
        roundtrip_compute<P, ALIGNED, BE, RNE, NT, U>(a, t, lut, lane, v);
        t += nwaves;
        if (t < a.ntiles) roundtrip_load<ALIGNED, U>(a, t, lane, v);
    }
}

// The fused round trip over a batch of slices (of one or several jobs) in ONE
// launch: the slices' tiles are numbered consecutively (tile_end[s] = tiles of
// slices 0..s), each wave finds its slice by a binary search over that
// wave-uniform table (kernel arguments, scalar loads) and runs the slice's
// own block geometry.  Slices start at any 4-byte offset (FIFO slices,
// pinned host tensors): the unaligned form, which streams at the aligned rate.
struct RoundTripBatchArgs {
    const float* in[SML_MAX_BATCH_SLICES];
    float* out[SML_MAX_BATCH_SLICES];
    uint64_t numel[SML_MAX_BATCH_SLICES];
    uint32_t tile_end[SML_MAX_BATCH_SLICES];
    uint32_t nslices;
    uint32_t W;
    uint32_t xcd;
};

template <int P, bool RNE, bool NT = false, int U = kU>
__global__ __launch_bounds__(kBlockThreads) void k_roundtrip_batch(RoundTripBatchArgs a) {
    __shared__ float lut[256];
    build_lut(lut, a.W);
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t nwaves = gridDim.x * kWavesPerBlock;
    const uint32_t ntiles = a.tile_end[a.nslices - 1];
    for (uint32_t t = (uint32_t)xcd_block(a.xcd) * kWavesPerBlock + wave_index(); t < ntiles; t += nwaves) {
        uint32_t lo = 0, hi = a.nslices - 1;             // first s with tile_end[s] > t
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (a.tile_end[mid] > t) hi = mid;
            else lo = mid + 1;
        }
        const uint32_t t0 = lo ? a.tile_end[lo - 1] : 0u;
        RoundTripArgs r;
        r.in = a.in[lo];
        r.out = a.out[lo];
        r.numel = a.numel[lo];
        r.nblocks = r.numel / P + (r.numel % P != 0);
        r.ntiles = a.tile_end[lo] - t0;
        r.payload = nullptr;
        r.exps_out = nullptr;
        r.W = a.W;
        r.xcd = a.xcd;
        roundtrip_tile<P, false, true, RNE, NT, U>(r, t - t0, lut, lane);
    }
}

// Word streams in the quantizer's tile shape (1024 words per wave, 16-B
// non-temporal loads, default-policy stores, XCD order, one-shot grid; any
// 4-byte alignment; in may alias out):
//  * K5 DummyBackend::ProcessPacket over the payload plane: per word bswap,
//    int32 wrap multiply by W, bswap (dummy_backend.cc:72-84); LE words skip
//    the swaps;
//  * INT32 path: byteswap (ppp.cc:158-190, 262-298).
struct LoopbackOp {
    uint32_t W;
    bool be;
    __device__ __forceinline__ uint32_t operator()(uint32_t q) const { return be ? bswap(bswap(q) * W) : q * W; }
};
struct BswapOp {
    __device__ __forceinline__ uint32_t operator()(uint32_t q) const { return bswap(q); }
};

// Measurement probe (not on the hot path): the same 1024-element tiles and
// the same access policy as the quantize kernel — non-temporal 16-B loads,
// and 16-B stores under K1's store policy for a plane of that size
// (non-temporal from g_nt_threshold bytes on, default policy below) — no
// arithmetic: the practical HBM ceiling the quantize kernel is compared
// against.
template <bool NTS, int U>
__global__ __launch_bounds__(kBlockThreads) void k_stream_copy(const u4* in, u4* out, uint64_t ntiles, uint32_t xcd) {
    struct { uint32_t xcd; } a{xcd};
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    constexpr uint64_t kVecs = tile_elems<U>() / 4;
    for (uint64_t t = xcd_block(a.xcd) * kWavesPerBlock + wave_index(); t < ntiles; t += nwaves) {
        u4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(in + t * kVecs + u * kWave + lane);
#pragma unroll
        for (int u = 0; u < U; u++) store_payload_as<NTS>(out + t * kVecs + u * kWave + lane, v[u]);
    }
}

// RDMA immediates: (msg_id & 0xFFFF) | exponent byte << 16 (rdma_worker_thread.cc:341-356).
__global__ __launch_bounds__(kBlockThreads) void k_rdma_imm(const int8_t* exps, uint64_t B, uint64_t total,
                                                            uint32_t* imm) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlockThreads;
    for (uint64_t m = (uint64_t)blockIdx.x * kBlockThreads + threadIdx.x; m < total; m += stride) {
        const uint32_t e = exps && m < B ? (uint32_t)(uint8_t)exps[m] : 0u;
        imm[m] = (uint32_t)(m & 0xFFFFu) | (e << 16);
    }
}

// Fault injection (sml_debug_stall): one wave that occupies its stream for
// `ticks` of the constant-rate wall clock, then exits — a kernel that does
// not finish within a caller's timeout, yet always ends on its own.
constexpr uint32_t kMaxStallMicros = 60u * 1000u * 1000u;
__global__ __launch_bounds__(64) void k_stall(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

__global__ void k_scale_lut(float* lut, uint32_t W) {
    lut[threadIdx.x] = scale_for(W, (int)(int8_t)(uint8_t)threadIdx.x);
}

// ------------------------------------------------------------ host side

// Dispatch tables: runtime (P, tile slices U, alignment, mode) -> template
// instance.  U is 1, 2 or 4 and at least P / 256 (quantize_common).
template <int P, bool ALIGNED, bool GLOBAL, bool BE, bool RNE>
static void launch_quant_u(uint32_t U, bool nts, dim3 grid, hipStream_t st, const QuantArgs& a) {
    if constexpr (P <= 256) {
        if (U == 1) {
            if (nts) k_quantize_pack<P, ALIGNED, GLOBAL, BE, RNE, 1, true><<<grid, kBlockThreads, 0, st>>>(a);
            else k_quantize_pack<P, ALIGNED, GLOBAL, BE, RNE, 1><<<grid, kBlockThreads, 0, st>>>(a);
            return;
        }
    }
    if constexpr (P <= 512) {
        if (U == 2) {
            if (nts) k_quantize_pack<P, ALIGNED, GLOBAL, BE, RNE, 2, true><<<grid, kBlockThreads, 0, st>>>(a);
            else k_quantize_pack<P, ALIGNED, GLOBAL, BE, RNE, 2><<<grid, kBlockThreads, 0, st>>>(a);
            return;
        }
    }
    if (nts) { k_quantize_pack<P, ALIGNED, GLOBAL, BE, RNE, 4, true><<<grid, kBlockThreads, 0, st>>>(a); return; }
    k_quantize_pack<P, ALIGNED, GLOBAL, BE, RNE, 4><<<grid, kBlockThreads, 0, st>>>(a);
}

template <bool ALIGNED, bool GLOBAL, bool BE, bool RNE>
static void launch_quant_p(uint32_t P, uint32_t U, bool nts, dim3 grid, hipStream_t st, const QuantArgs& a) {
    switch (P) {
        case 64:   launch_quant_u<64, ALIGNED, GLOBAL, BE, RNE>(U, nts, grid, st, a); break;
        case 128:  launch_quant_u<128, ALIGNED, GLOBAL, BE, RNE>(U, nts, grid, st, a); break;
        case 256:  launch_quant_u<256, ALIGNED, GLOBAL, BE, RNE>(U, nts, grid, st, a); break;
        case 512:  launch_quant_u<512, ALIGNED, GLOBAL, BE, RNE>(U, nts, grid, st, a); break;
        default:   launch_quant_u<1024, ALIGNED, GLOBAL, BE, RNE>(U, nts, grid, st, a); break;
    }
}

// Slices per K1/K2/K3 tile: 4 (1024-element tiles), 2 or 1 (never below
// P / 256), or 0 = the default, 2 for every kernel (sml_set_quantize_tile_slices).
// Final kernels (early loads, sc1 nt stores; profiles/r04/ab_slices_final.json,
// 4 cold buckets, interleaved medians): 2-slice tiles against 4 at 256 MiB
// K1 -3.1 %, K3 -2.0 %, K2 -3.2 % time (K1 -4.9 % at 128 MiB).  Before the
// early loads and sc1 (round 4's first sweep), measured with non-temporal payload stores
// on the bench workload, steps cycling 4 buckets (round 4,
// profiles/r04/ab_slices_nt.json, interleaved medians): K1 with 2-slice tiles
// +1.3 / +0.6 / +3.8 / +0.9 % at 128 / 256 / 512 / 1024 MiB, K3 -2.8 % and
// K2 -2.6 % at 256 MiB; 1-slice tiles lose everywhere (K1 -3 %, K2 -35 %:
// one 1 KiB load in flight per wave is latency-bound).  Round 2's sweep ran
// before the non-temporal stores and had 2-slice K1 level cold.
static std::atomic<uint32_t> g_quant_slices{0};

// Payload planes (and K4 / round-trip fp32 outputs) of at least this many
// bytes take non-temporal stores (sml_set_payload_nt_threshold; UINT64_MAX =
// never, 0 = always).  Measured on cold HBM — steps cycling distinct buckets,
// the pattern of a real job where a plane is written once and handed on
// (profiles/r03/ab_cold_policy*.json, interleaved medians): non-temporal
// stores win at 64 / 128 / 256 MiB planes for K1 (+4.1 / +3.5 / +4.6 %), K4
// (+5.6 / +6.3 / +4.5 %) and the fused round trip (+4.2 / +3.1 / +3.5 %).
// Default-policy stores win only when ONE plane is rewritten step after step
// (it then stays in the 256 MiB Infinity Cache: K1 7.13 vs 6.31 TB/s at
// 256 MiB, 6.54 vs 6.09 at 128 MiB; level at 64 MiB).  So planes from a
// quarter of the Infinity Cache on stream non-temporally; smaller ones (a
// framework's 25 MiB gradient buckets) keep the default policy, so their
// next reader can find them in the cache.  Bytes are identical either way.
std::atomic<uint64_t> g_nt_threshold{64ull << 20};

// Slices per K4 / fused round-trip tile: 4 or 2 (sml_set_stream_tile_slices;
// 0 = the default, 2 for both — a round-trip tile holds whole packets, so
// P = 1024 keeps 4.  Final kernels, profiles/r04/ab_stream_slices_final.json:
// 2 against 4 at 256 / 128 MiB, K4 -0.8 / -1.9 %, the round trip -3.4 / -3.6 %
// time; round 4's first sweep, before the early loads and sc1 stores, had
// the round trip level).
static std::atomic<uint32_t> g_stream_slices{0};

static uint32_t stream_slices(uint32_t dflt) {
    const uint32_t want = g_stream_slices.load(std::memory_order_relaxed);
    return want ? want : dflt;
}

static uint32_t quant_slices(uint32_t P) {
    const uint32_t need = P > 256 ? P / 256 : 1;
    uint32_t want = g_quant_slices.load(std::memory_order_relaxed);
    if (want == 0) want = 2u;
    return want > need ? want : need;
}

template <bool ALIGNED, bool GLOBAL, bool BE>
static void launch_quant_r(bool rne, uint32_t P, uint32_t U, bool nts, dim3 g, hipStream_t st, const QuantArgs& a) {
    if (rne) launch_quant_p<ALIGNED, GLOBAL, BE, true>(P, U, nts, g, st, a);
    else launch_quant_p<ALIGNED, GLOBAL, BE, false>(P, U, nts, g, st, a);
}

template <bool ALIGNED, bool GLOBAL>
static void launch_quant_b(bool be, bool rne, uint32_t P, uint32_t U, bool nts, dim3 g, hipStream_t st,
                           const QuantArgs& a) {
    if (be) launch_quant_r<ALIGNED, GLOBAL, true>(rne, P, U, nts, g, st, a);
    else launch_quant_r<ALIGNED, GLOBAL, false>(rne, P, U, nts, g, st, a);
}

template <bool ALIGNED, bool BE, bool RCP, bool NT, int U>
static void launch_deq_pn(uint32_t P, dim3 grid, hipStream_t st, const DequantArgs& a) {
    switch (P) {
        case 64:   k_dequantize<64, ALIGNED, BE, RCP, NT, U><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 128:  k_dequantize<128, ALIGNED, BE, RCP, NT, U><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 256:  k_dequantize<256, ALIGNED, BE, RCP, NT, U><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 512:  k_dequantize<512, ALIGNED, BE, RCP, NT, U><<<grid, kBlockThreads, 0, st>>>(a); break;
        default:   k_dequantize<1024, ALIGNED, BE, RCP, NT, U><<<grid, kBlockThreads, 0, st>>>(a); break;
    }
}

template <bool ALIGNED, bool BE, bool RCP>
static void launch_deq_p(uint32_t P, uint32_t U, bool nt, dim3 grid, hipStream_t st, const DequantArgs& a) {
    if (U == 2) {
        if (nt) launch_deq_pn<ALIGNED, BE, RCP, true, 2>(P, grid, st, a);
        else launch_deq_pn<ALIGNED, BE, RCP, false, 2>(P, grid, st, a);
        return;
    }
    if (nt) launch_deq_pn<ALIGNED, BE, RCP, true, 4>(P, grid, st, a);
    else launch_deq_pn<ALIGNED, BE, RCP, false, 4>(P, grid, st, a);
}

template <bool ALIGNED, bool BE>
static void launch_deq_w(uint32_t P, uint32_t U, bool nt, dim3 grid, hipStream_t st, const DequantArgs& a) {
    if ((a.W & (a.W - 1)) == 0) launch_deq_p<ALIGNED, BE, true>(P, U, nt, grid, st, a);
    else launch_deq_p<ALIGNED, BE, false>(P, U, nt, grid, st, a);
}

template <bool ALIGNED, bool BE, bool RNE, bool NT, int U>
static void launch_rt_pn(uint32_t P, dim3 grid, hipStream_t st, const RoundTripArgs& a) {
    switch (P) {
        case 64:   k_roundtrip<64, ALIGNED, BE, RNE, NT, U><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 128:  k_roundtrip<128, ALIGNED, BE, RNE, NT, U><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 256:  k_roundtrip<256, ALIGNED, BE, RNE, NT, U><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 512:  k_roundtrip<512, ALIGNED, BE, RNE, NT, U><<<grid, kBlockThreads, 0, st>>>(a); break;
        default:   k_roundtrip<1024, ALIGNED, BE, RNE, NT, 4><<<grid, kBlockThreads, 0, st>>>(a); break;   // a tile holds the packet
    }
}

template <bool ALIGNED, bool BE, bool RNE>
static void launch_rt_p(uint32_t P, uint32_t U, bool nt, dim3 grid, hipStream_t st, const RoundTripArgs& a) {
    if (U == 2) {
        if (nt) launch_rt_pn<ALIGNED, BE, RNE, true, 2>(P, grid, st, a);
        else launch_rt_pn<ALIGNED, BE, RNE, false, 2>(P, grid, st, a);
        return;
    }
    if (nt) launch_rt_pn<ALIGNED, BE, RNE, true, 4>(P, grid, st, a);
    else launch_rt_pn<ALIGNED, BE, RNE, false, 4>(P, grid, st, a);
}

template <bool RNE, bool NT>
static void launch_rtb_pn(uint32_t P, uint32_t U, dim3 grid, hipStream_t st, const RoundTripBatchArgs& a) {
    // a tile holds whole packets: P = 1024 runs 4 slices
    if (U == 2) {
        switch (P) {
            case 64:   k_roundtrip_batch<64, RNE, NT, 2><<<grid, kBlockThreads, 0, st>>>(a); return;
            case 128:  k_roundtrip_batch<128, RNE, NT, 2><<<grid, kBlockThreads, 0, st>>>(a); return;
            case 256:  k_roundtrip_batch<256, RNE, NT, 2><<<grid, kBlockThreads, 0, st>>>(a); return;
            case 512:  k_roundtrip_batch<512, RNE, NT, 2><<<grid, kBlockThreads, 0, st>>>(a); return;
            default:   break;
        }
    }
    switch (P) {
        case 64:   k_roundtrip_batch<64, RNE, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 128:  k_roundtrip_batch<128, RNE, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 256:  k_roundtrip_batch<256, RNE, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 512:  k_roundtrip_batch<512, RNE, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
        default:   k_roundtrip_batch<1024, RNE, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
    }
}

template <bool RNE>
static void launch_rtb_p(uint32_t P, uint32_t U, bool nt, dim3 grid, hipStream_t st, const RoundTripBatchArgs& a) {
    if (nt) launch_rtb_pn<RNE, true>(P, U, grid, st, a);
    else launch_rtb_pn<RNE, false>(P, U, grid, st, a);
}

template <bool ALIGNED>
static void launch_rt_a(bool be, bool rne, bool nt, uint32_t P, uint32_t U, dim3 g, hipStream_t st,
                        const RoundTripArgs& a) {
    if (be) { if (rne) launch_rt_p<ALIGNED, true, true>(P, U, nt, g, st, a); else launch_rt_p<ALIGNED, true, false>(P, U, nt, g, st, a); }
    else    { if (rne) launch_rt_p<ALIGNED, false, true>(P, U, nt, g, st, a); else launch_rt_p<ALIGNED, false, false>(P, U, nt, g, st, a); }
}

}  // namespace sml

using namespace sml;

extern "C" {

int sml_abi_version(void) { return SML_ABI_VERSION; }

const char* sml_status_string(sml_status_t s) {
    switch (s) {
        case SML_OK: return "SML_OK";
        case SML_ERR_INVALID_ARG: return "SML_ERR_INVALID_ARG";
        case SML_ERR_UNSUPPORTED: return "SML_ERR_UNSUPPORTED";
        case SML_ERR_ALIGNMENT: return "SML_ERR_ALIGNMENT";
        case SML_ERR_HIP: return "SML_ERR_HIP";
    }
    return "SML_ERR_UNKNOWN";
}

const char* sml_last_error(void) { return g_last_error; }

uint32_t sml_set_grid_limit(uint32_t max_workgroups) {
    return g_grid_limit.exchange(max_workgroups);
}

uint32_t sml_set_xcd_chunk(uint32_t chunk) {
    return g_xcd_chunk.exchange(chunk);
}

uint64_t sml_set_payload_nt_threshold(uint64_t bytes) { return g_nt_threshold.exchange(bytes); }

uint32_t sml_set_stream_tile_slices(uint32_t slices) {
    return g_stream_slices.exchange(slices == 2 || slices == 4 ? slices : 0u);
}

uint32_t sml_set_quantize_tile_slices(uint32_t slices) {
    return g_quant_slices.exchange(slices == 1 || slices == 2 || slices == 4 ? slices : 0u);
}

uint64_t sml_num_blocks(uint64_t numel, uint32_t packet_numel) {
    if (packet_numel == 0) return 0;
    // ceil(numel*4 / (P*4)) of ppp.cc:56-57, without the byte-count overflow
    return numel / packet_numel + (numel % packet_numel != 0);
}

sml_status_t sml_scale_lut(uint16_t num_workers, float lut[256]) {
    if (num_workers == 0 || !lut) return SML_ERR_INVALID_ARG;
    for (int i = 0; i < 256; i++) {
        int e = (int)(int8_t)(uint8_t)i;
        float denom = (float)num_workers * powf(2.0f, (float)e);
        lut[i] = (float)((double)2147483647 / (double)denom);
    }
    return SML_OK;
}

sml_status_t sml_scale_lut_device(uint16_t num_workers, float* d_lut, void* stream) {
    if (num_workers == 0 || !d_lut) return SML_ERR_INVALID_ARG;
    k_scale_lut<<<1, 256, 0, (hipStream_t)stream>>>(d_lut, num_workers);
    return launch_check();
}

static sml_status_t quantize_common(const float* d_in, uint64_t numel, uint32_t P, uint16_t W,
                                    const int8_t* d_gexp, int32_t* d_payload, int8_t* d_exps_out,
                                    uint32_t flags, void* stream) {
    if (!valid_packet(P)) return SML_ERR_UNSUPPORTED;
    if (numel == 0) return SML_OK;
    if (!d_in || !aligned4(d_in)) return SML_ERR_INVALID_ARG;
    if (d_payload && !aligned16(d_payload)) return SML_ERR_ALIGNMENT;
    QuantArgs a;
    const uint32_t U = quant_slices(P);
    // XCD runs keep their byte length (C workgroups of 4 U-slice tiles)
    a.xcd = g_xcd_chunk.load(std::memory_order_relaxed) * (4 / U);
    a.in = d_in;
    a.numel = numel;
    a.nblocks = sml_num_blocks(numel, P);
    const uint64_t te = 256ull * U;
    a.ntiles = (a.nblocks * P + te - 1) / te;
    a.gexp = d_gexp;
    a.payload = reinterpret_cast<u4*>(d_payload);
    a.exps_out = d_gexp ? nullptr : d_exps_out;
    a.W = W;
    dim3 grid(grid_for_tiles(a.ntiles));
    hipStream_t st = (hipStream_t)stream;
    const bool al = aligned16(d_in), be = !(flags & SML_FLAG_PAYLOAD_LE), rne = flags & SML_FLAG_ROUND_RNE;
    // payload store policy by plane size
    const bool nts = d_payload && 4 * numel >= g_nt_threshold.load(std::memory_order_relaxed);
    if (d_gexp) {
        if (al) launch_quant_b<true, true>(be, rne, P, U, nts, grid, st, a);
        else launch_quant_b<false, true>(be, rne, P, U, nts, grid, st, a);
    } else {
        if (al) launch_quant_b<true, false>(be, rne, P, U, nts, grid, st, a);
        else launch_quant_b<false, false>(be, rne, P, U, nts, grid, st, a);
    }
    return launch_check();
}

sml_status_t sml_exponents(const float* d_in, uint64_t numel, uint32_t packet_numel,
                           int8_t* d_exps, void* stream) {
    if (numel && !d_exps) return SML_ERR_INVALID_ARG;
    return quantize_common(d_in, numel, packet_numel, 1, nullptr, nullptr, d_exps, 0, stream);
}

sml_status_t sml_quantize_pack(const float* d_in, uint64_t numel, uint32_t packet_numel,
                               uint16_t num_workers, const int8_t* d_global_exps,
                               int32_t* d_payload, int8_t* d_exps_out,
                               uint32_t flags, void* stream) {
    if (num_workers == 0) return SML_ERR_INVALID_ARG;
    if (numel && !d_payload) return SML_ERR_INVALID_ARG;
    if (d_global_exps && d_exps_out && d_exps_out != d_global_exps) return SML_ERR_INVALID_ARG;
    return quantize_common(d_in, numel, packet_numel, num_workers, d_global_exps, d_payload,
                           d_exps_out, flags, stream);
}

sml_status_t sml_dequantize(const int32_t* d_payload, const int8_t* d_exps, uint64_t numel,
                            uint32_t packet_numel, uint16_t num_workers, float* d_out,
                            uint32_t flags, void* stream) {
    if (!valid_packet(packet_numel)) return SML_ERR_UNSUPPORTED;
    if (num_workers == 0) return SML_ERR_INVALID_ARG;
    if (numel == 0) return SML_OK;
    if (!d_payload || !d_exps || !d_out || !aligned4(d_out)) return SML_ERR_INVALID_ARG;
    if (!aligned16(d_payload)) return SML_ERR_ALIGNMENT;
    DequantArgs a;
    const uint32_t U = stream_slices(2);   // measured: 2-slice tiles +0.6 / +2.8 / +3.3 % at 128 / 256 / 512 MiB
    a.xcd = g_xcd_chunk.load(std::memory_order_relaxed) * (4 / U);   // XCD runs keep their byte length
    a.payload = reinterpret_cast<const u4*>(d_payload);
    a.exps = d_exps;
    a.out = d_out;
    a.numel = numel;
    a.ntiles = (numel + 256 * U - 1) / (256 * U);
    a.W = num_workers;
    dim3 grid(grid_for_tiles(a.ntiles));
    hipStream_t st = (hipStream_t)stream;
    const bool al = aligned16(d_out), be = !(flags & SML_FLAG_PAYLOAD_LE);
    const bool nt = 4 * numel >= g_nt_threshold.load(std::memory_order_relaxed);   // output plane past the Infinity Cache
    if (al) { if (be) launch_deq_w<true, true>(packet_numel, U, nt, grid, st, a); else launch_deq_w<true, false>(packet_numel, U, nt, grid, st, a); }
    else    { if (be) launch_deq_w<false, true>(packet_numel, U, nt, grid, st, a); else launch_deq_w<false, false>(packet_numel, U, nt, grid, st, a); }
    return launch_check();
}

sml_status_t sml_roundtrip_loopback(const float* d_in, float* d_out, uint64_t numel,
                                    uint32_t packet_numel, uint16_t num_workers,
                                    int32_t* d_payload, int8_t* d_exps_out,
                                    uint32_t flags, void* stream) {
    if (!valid_packet(packet_numel)) return SML_ERR_UNSUPPORTED;
    if (num_workers == 0) return SML_ERR_INVALID_ARG;
    if (numel == 0) return SML_OK;
    if (!d_in || !d_out || !aligned4(d_in) || !aligned4(d_out)) return SML_ERR_INVALID_ARG;
    if (d_payload && !aligned16(d_payload)) return SML_ERR_ALIGNMENT;
    RoundTripArgs a;
    // a tile holds whole packets: P = 1024 needs 4 slices
    const uint32_t U = packet_numel > 512 ? 4u : stream_slices(2);
    a.xcd = g_xcd_chunk.load(std::memory_order_relaxed) * (4 / U);
    a.in = d_in;
    a.out = d_out;
    a.numel = numel;
    a.nblocks = sml_num_blocks(numel, packet_numel);
    a.ntiles = (a.nblocks * packet_numel + 256 * U - 1) / (256 * U);
    a.payload = reinterpret_cast<u4*>(d_payload);
    a.exps_out = d_exps_out;
    a.W = num_workers;
    dim3 grid(grid_for_tiles(a.ntiles));
    hipStream_t st = (hipStream_t)stream;
    // in and out share the slice offset, so one alignment test covers both
    // unless the caller passed differently aligned buffers.
    const bool al = aligned16(d_in) && aligned16(d_out);
    const bool be = !(flags & SML_FLAG_PAYLOAD_LE), rne = flags & SML_FLAG_ROUND_RNE;
    const bool nt = 4 * numel >= g_nt_threshold.load(std::memory_order_relaxed);   // output plane past the Infinity Cache
    if (al) launch_rt_a<true>(be, rne, nt, packet_numel, U, grid, st, a);
    else launch_rt_a<false>(be, rne, nt, packet_numel, U, grid, st, a);
    return launch_check();
}

sml_status_t sml_roundtrip_loopback_batch(const sml_slice* slices, uint32_t num_slices, uint32_t packet_numel,
                                          uint16_t num_workers, uint32_t flags, void* stream) {
    if (!valid_packet(packet_numel)) return SML_ERR_UNSUPPORTED;
    if (num_workers == 0 || num_slices > SML_MAX_BATCH_SLICES || (num_slices && !slices)) return SML_ERR_INVALID_ARG;
    RoundTripBatchArgs a;
    // tile slices (P = 1024: 4): the single-slice round trip's 2 — against 4
    // on 4 cold jobs: a 256 MiB job as 4 FIFO slices 86.22 -> 85.86 us, 4 x
    // 25 MiB buckets 36.10 -> 35.32 us (profiles/r04/ab_batch_slices.json).
    const uint32_t U = packet_numel > 512 ? 4u : 2u;
    const uint64_t tile = (uint64_t)U * kWave * 4;
    a.xcd = g_xcd_chunk.load(std::memory_order_relaxed) * (4 / U);   // XCD runs keep their byte length
    a.W = num_workers;
    a.nslices = 0;
    uint64_t tiles = 0;
    for (uint32_t i = 0; i < num_slices; i++) {
        const sml_slice& sl = slices[i];
        if (sl.numel == 0) continue;                      // empty slices touch nothing
        if (!sl.in || !sl.out || !aligned4(sl.in) || !aligned4(sl.out)) return SML_ERR_INVALID_ARG;
        tiles += (sml_num_blocks(sl.numel, packet_numel) * packet_numel + tile - 1) / tile;
        if (tiles > 0xFFFFFFFFull) return SML_ERR_UNSUPPORTED;
        a.in[a.nslices] = sl.in;
        a.out[a.nslices] = sl.out;
        a.numel[a.nslices] = sl.numel;
        a.tile_end[a.nslices] = (uint32_t)tiles;
        a.nslices++;
    }
    if (a.nslices == 0) return SML_OK;
    if (a.nslices == 1)   // one slice: the single-slice kernel (aligned form when the slice allows it)
        return sml_roundtrip_loopback(a.in[0], a.out[0], a.numel[0], packet_numel, num_workers, nullptr, nullptr,
                                      flags & SML_FLAG_ROUND_RNE, stream);
    const dim3 grid(grid_for_tiles(tiles));
    hipStream_t st = (hipStream_t)stream;
    // the outputs of the whole batch past the Infinity Cache: non-temporal stores
    uint64_t out_bytes = 0;
    for (uint32_t i = 0; i < a.nslices; i++) out_bytes += 4 * a.numel[i];
    const bool nt = out_bytes >= g_nt_threshold.load(std::memory_order_relaxed);
    if (flags & SML_FLAG_ROUND_RNE) launch_rtb_p<true>(packet_numel, U, nt, grid, st, a);
    else launch_rtb_p<false>(packet_numel, U, nt, grid, st, a);
    return launch_check();
}

sml_status_t sml_rdma_imm(const int8_t* d_exps, uint64_t B, uint32_t batch_max, uint32_t* d_imm, void* stream) {
    if (B == 0) return SML_OK;
    // a FLOAT32 slice needs its exponent plane: a null one is an error, not
    // an INT32 slice (sml_rdma_imm_int32 is that)
    if (!d_imm || !d_exps || batch_max == 0) return SML_ERR_INVALID_ARG;
    const uint64_t total = B + (B < batch_max ? B : batch_max);
    k_rdma_imm<<<grid_for_vec(total), kBlockThreads, 0, (hipStream_t)stream>>>(d_exps, B, total, d_imm);
    return launch_check();
}

sml_status_t sml_rdma_imm_int32(uint64_t B, uint32_t* d_imm, void* stream) {
    if (B == 0) return SML_OK;
    if (!d_imm) return SML_ERR_INVALID_ARG;
    // B messages (no extra batch, ppp.cc:65-67), byte 2 untouched (0)
    k_rdma_imm<<<grid_for_vec(B), kBlockThreads, 0, (hipStream_t)stream>>>(nullptr, B, B, d_imm);
    return launch_check();
}

sml_status_t sml_debug_stall(uint32_t microseconds, void* stream) {
    if (microseconds == 0) return SML_OK;
    if (microseconds > kMaxStallMicros) return SML_ERR_INVALID_ARG;
    int dev = 0, khz = 0;
    sml_status_t s = hip_check(hipGetDevice(&dev));
    if (s == SML_OK) s = hip_check(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    if (s != SML_OK) return s;
    if (khz <= 0) return SML_ERR_HIP;
    k_stall<<<1, 64, 0, (hipStream_t)stream>>>((uint64_t)microseconds * (uint64_t)khz / 1000u);
    return launch_check();
}

sml_status_t sml_stream_copy(const void* d_in, void* d_out, uint64_t bytes, void* stream) {
    if (bytes == 0) return SML_OK;
    if (!d_in || !d_out || !aligned16(d_in) || !aligned16(d_out) || bytes % (kTileElems * 4)) return SML_ERR_ALIGNMENT;
    // K1's tile shape (its slices per tile at P = 256) and store policy for an
    // output plane of `bytes` (sml_quantize_pack)
    const uint32_t U = quant_slices(256);
    const uint64_t ntiles = bytes / (256 * U * 4);
    const uint32_t xcd = g_xcd_chunk.load(std::memory_order_relaxed) * (4 / U);
    auto in = reinterpret_cast<const u4*>(d_in);
    auto out = reinterpret_cast<u4*>(d_out);
    const bool nts = bytes >= g_nt_threshold.load(std::memory_order_relaxed);
    const dim3 grid(grid_for_tiles(ntiles));
    hipStream_t st = (hipStream_t)stream;
#define SML_COPY(U_)                                                                     \
    if (nts) k_stream_copy<true, U_><<<grid, kBlockThreads, 0, st>>>(in, out, ntiles, xcd); \
    else k_stream_copy<false, U_><<<grid, kBlockThreads, 0, st>>>(in, out, ntiles, xcd);
    if (U == 1) { SML_COPY(1) } else if (U == 2) { SML_COPY(2) } else { SML_COPY(4) }
#undef SML_COPY
    return launch_check();
}

sml_status_t sml_bswap_i32(const int32_t* d_in, int32_t* d_out, uint64_t numel, void* stream) {
    if (numel == 0) return SML_OK;
    if (!d_in || !d_out || !aligned4(d_in) || !aligned4(d_out)) return SML_ERR_INVALID_ARG;
    const uint64_t ntiles = (numel + kTileElems - 1) / kTileElems;
    k_words<<<grid_for_tiles(ntiles), kBlockThreads, 0, (hipStream_t)stream>>>(
        reinterpret_cast<const uint32_t*>(d_in), reinterpret_cast<uint32_t*>(d_out), numel,
        g_xcd_chunk.load(std::memory_order_relaxed), BswapOp{});
    return launch_check();
}

sml_status_t sml_loopback_aggregate(int32_t* d_payload, uint64_t count, uint16_t num_workers,
                                    uint32_t flags, void* stream) {
    if (num_workers == 0) return SML_ERR_INVALID_ARG;
    if (count == 0) return SML_OK;
    if (!d_payload) return SML_ERR_INVALID_ARG;
    if (!aligned16(d_payload) || (count & 3u)) return SML_ERR_ALIGNMENT;
    const uint64_t ntiles = (count + kTileElems - 1) / kTileElems;
    uint32_t* p = reinterpret_cast<uint32_t*>(d_payload);
    k_words<<<grid_for_tiles(ntiles), kBlockThreads, 0, (hipStream_t)stream>>>(
        p, p, count, g_xcd_chunk.load(std::memory_order_relaxed),
        LoopbackOp{num_workers, !(flags & SML_FLAG_PAYLOAD_LE)});
    return launch_check();
}

}  // extern "C"
