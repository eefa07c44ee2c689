// sml_frames.hip — DPDK wire frames on gfx950: the transmit
// side (BuildPacket + PreprocessSingle for every packet of a slice,
// client_lib/src/backends/dpdk/dpdk_worker_thread_utils.inc:42-135) and the
// receive side (DpdkWorkerThread's rx loop, dpdk_worker_thread.cc:300-345,
// with PostprocessSingle per accepted frame), and their C-ABI entry points.
#include "sml_host.h"

namespace sml {

// ---------------------------------------------------------- DPDK frames

struct FrameArgs {
    const float* in;
    uint64_t numel;
    uint64_t nblocks;       // B
    uint64_t ntiles;        // ceil(B*P / 1024)
    uint64_t b;             // extra-batch size = min(batch_max, B)
    const int8_t* gexp;     // global exponents or nullptr
    uint8_t* frames;        // B + b frames, 4-byte aligned
    uint64_t stride;        // bytes between frames, multiple of 4
    uint32_t W;
    uint32_t xcd;           // xcd_block chunk (0 = plain order)
    uint32_t pool_start, pool_shift, mop;
    uint32_t hdr[11];       // frame bytes 0..43: Eth, IPv4, UDP, job_type_size, short_job_id
};

// PktId2PoolIndex, dpdk_worker_thread_utils.inc:42-52.
__device__ __forceinline__ uint32_t pool_index(uint64_t p, const FrameArgs& a) {
    const uint32_t i = (uint32_t)((p + a.pool_shift) % (2ull * a.mop));
    return i < a.mop ? ((a.pool_start + i) & 0xffffu) : (((a.pool_start + (i - a.mop)) | 0x8000u) & 0xffffu);
}

// Lanes 0..12 write the 52 header bytes of frame p (one dword each):
// dwords 0-10 constant, 11 = pkt_id (host order), 12 = pool index (BE16),
// exponent byte, zero byte.  (Extra-batch frames; the bulk of the headers is
// written lane-parallel by k_quantize_frames.)
__device__ __forceinline__ void write_frame_header(const FrameArgs& a, uint64_t p, int lane, uint32_t exp_byte) {
    if (lane > 12) return;
    uint32_t dw = a.hdr[0];
#pragma unroll
    for (int i = 1; i < 11; i++) dw = lane == i ? a.hdr[i] : dw;
    if (lane == 11) dw = (uint32_t)p;
    if (lane == 12) {
        const uint32_t pool = pool_index(p, a);
        dw = (pool >> 8) | ((pool & 0xffu) << 8) | ((exp_byte & 0xffu) << 16);
    }
    *reinterpret_cast<uint32_t*>(a.frames + p * a.stride + 4 * lane) = dw;
}

// Fused quantize + pack into DPDK frames (BuildPacket + PreprocessSingle for
// every packet of the slice, dpdk_worker_thread_utils.inc:67-135 + ppp.cc:69-156).
//
// Frame f carries the exponent of block f (f < B) in header dword 12 (pool
// index BE16, exponent byte, zero byte) and the payload of block f - b.  The
// wave of block k therefore writes:
//  * frame k + b: header dwords 0-11 and the payload — one wave writes all
//    of the frame but dword 12 (and dword 12 too once k + b >= B: those
//    frames carry exponent 0);
//  * dword 12 of frame k (k >= b), or the whole of extra-batch frame k
//    (k < b: header with this exponent, zero payload).
// One dword store instruction covers 4 frames: lane l < 48 writes dword
// l % 12 of payload frame l / 12, lanes 48-51 write dword 12 of the 4
// exponent frames.  Constant dwords are picked once per wave; the pool index
// (PktId2PoolIndex) costs one 64-bit modulo per tile.
__device__ __forceinline__ uint32_t pool_dword(const FrameArgs& a, uint32_t i, uint32_t exp_byte) {
    const uint32_t pool = i < a.mop ? ((a.pool_start + i) & 0xffffu) : (((a.pool_start + (i - a.mop)) | 0x8000u) & 0xffffu);
    return (pool >> 8) | ((pool & 0xffu) << 8) | ((exp_byte & 0xffu) << 16);
}

// Held to 8 waves per SIMD: left to itself hipcc gives it 106 SGPRs, which
// caps it at 7; at 8 (a few SGPRs live in VGPR lanes, no scratch) the
// 256 MiB bucket's frames take 4 % less time (profiles/r02c/ab_frames_occupancy.json).
// The rx apply pass measured 1.6 % slower the same way and is left alone.
// NTS: the payload words take non-temporal stores (frames in device memory
// from the non-temporal threshold on).  Measured on cold frame sets (4
// cycled, 256 MiB bucket, profiles/r04/ab_frames_nt.json): 98.1 -> 86.4 us;
// non-temporal header dwords as well: 109.6 us (partial-line stores), so
// headers keep the default policy.
// I32: an INT32 job slice (DataType::INT32): no extra batch (a.b = 0), so
// frame f carries block f; its payload is htonl of the block's words
// (ppp.cc:158-190) and its exponent byte 0 — the same tile walk, no scale.
template <int P, bool ALIGNED, bool GLOBAL, bool NTS = false, bool I32 = false>
__global__ __attribute__((amdgpu_waves_per_eu(8, 8))) __launch_bounds__(kBlockThreads)
void k_quantize_frames(FrameArgs a) {
    __shared__ float lut[256];
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t padded = a.nblocks * P;
    constexpr int kPk = kTileElems / P;                   // packets per tile
    constexpr int kLanesPerPk = P / 4 < kWave ? P / 4 : kWave;
    const int hd = lane % 12;                              // header dword of lanes 0..47
    const int hj = lane < 48 ? lane / 12 : lane - 48;      // frame (of 4) of lanes 0..51
    uint32_t hconst = a.hdr[0];
#pragma unroll
    for (int i = 1; i < 11; i++) hconst = hd == i ? a.hdr[i] : hconst;
    const uint32_t m2 = 2u * a.mop;
    QuantArgs qa;                                          // reuse the K1 tile loader
    qa.in = a.in;
    qa.numel = a.numel;
    // As K1: the first tile's loads go out before the scale table is built.
    uint64_t t = xcd_block(a.xcd) * kWavesPerBlock + wave_index();
    f4 v[kU];
    if (t < a.ntiles) load_tile<ALIGNED>(qa, t * kTileElems, lane, v);
    if constexpr (!I32) build_lut(lut, a.W);
    for (bool first = true; t < a.ntiles; t += nwaves, first = false) {
        const uint64_t base = t * kTileElems;
        const uint64_t pk0 = base / P;                     // first block of the tile
        if (!first) load_tile<ALIGNED>(qa, base, lane, v); // later tiles (grid-stride)
        int eloc[kU];
        if constexpr (I32) {
#pragma unroll
            for (int u = 0; u < kU; u++) eloc[u] = 0;
        } else {
            tile_exponents<P>(v, eloc);
        }
        // exponent of packet j of the tile: slice j*P/256, lane (j*P/4) % 64
        uint32_t ej[kPk];
#pragma unroll
        for (int j = 0; j < kPk; j++) {
            const int u = (j * P) / 256;
            ej[j] = 0;
#pragma unroll
            for (int uu = 0; uu < kU; uu++)
                if (uu == u) ej[j] = (uint32_t)__builtin_amdgcn_readlane(eloc[uu], (j * kLanesPerPk) % kWave);
        }
        const uint32_t r = (uint32_t)((pk0 + a.pool_shift) % m2);   // pool slot of frame pk0
        const bool extra = pk0 < a.b;                               // wave-uniform, first b / kPk tiles
#pragma unroll
        for (int j0 = 0; j0 < kPk; j0 += 4) {
            const int j = j0 + hj;
            if (lane < 48) {
                if (j < kPk && pk0 + j < a.nblocks) {
                    const uint64_t f = pk0 + j + a.b;
                    *reinterpret_cast<uint32_t*>(a.frames + f * a.stride + 4 * hd) = hd == 11 ? (uint32_t)f : hconst;
                }
            } else if (lane < 52 && !extra) {
                if (j < kPk && pk0 + j < a.nblocks) {
                    uint32_t e = 0;
#pragma unroll
                    for (int jj = 0; jj < kPk; jj++) e = j == jj ? ej[jj] : e;
                    *reinterpret_cast<uint32_t*>(a.frames + (pk0 + j) * a.stride + 48) = pool_dword(a, (r + (uint32_t)j) % m2, e);
                }
            }
        }
        if (__builtin_expect(pk0 + kPk + a.b > a.nblocks, 0)) {
            // tail: payload frames at or past B carry exponent 0; their dword 12 is ours
            if (lane < kPk && pk0 + lane < a.nblocks && pk0 + lane + a.b >= a.nblocks) {
                const uint64_t f = pk0 + lane + a.b;
                *reinterpret_cast<uint32_t*>(a.frames + f * a.stride + 48) =
                    pool_dword(a, (uint32_t)((f + a.pool_shift) % m2), 0u);
            }
        }
        if (__builtin_expect(extra, 0)) {
            // extra-batch frames: header with this tile's exponent, zero payload; all ours
#pragma unroll
            for (int j = 0; j < kPk; j++) {
                const uint64_t pk = pk0 + j;
                if (pk >= a.nblocks) break;
                if (pk < a.b) {
                    write_frame_header(a, pk, lane, ej[j]);
                    uint32_t* pl = reinterpret_cast<uint32_t*>(a.frames + pk * a.stride + 52);
                    for (int i = lane; i < P / 4; i += kWave) *reinterpret_cast<u4a*>(pl + 4 * i) = u4a{0u, 0u, 0u, 0u};
                } else if (lane == 0) {
                    *reinterpret_cast<uint32_t*>(a.frames + pk * a.stride + 48) =
                        pool_dword(a, (uint32_t)((pk + a.pool_shift) % m2), ej[j]);
                }
            }
        }
        // payloads
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4;
            if (idx >= padded) continue;
            const uint64_t k = idx / P;
            u4 q;
            if constexpr (I32) {
                // the words as loaded (whole-vector bit cast: hipcc's bit cast of one
                // vector component returned component x for every component)
                q = __builtin_bit_cast(u4, v[u]);
            } else {
                int e = eloc[u];
                if constexpr (GLOBAL) e = a.gexp[k];
                q = quantize4<false>(v[u], lut[(uint8_t)e], idx, 0);
            }
            uint32_t* dst = reinterpret_cast<uint32_t*>(a.frames + (k + a.b) * a.stride + 52) + (idx - k * P);
            const u4a wq{bswap(q.x), bswap(q.y), bswap(q.z), bswap(q.w)};
            if constexpr (NTS) SML_NT_STORE16_UNALIGNED(wq, reinterpret_cast<u4a*>(dst));
            else *reinterpret_cast<u4a*>(dst) = wq;
        }
    }
}

// ------------------------------------------------- DPDK frames, receive side
//
// The rx bitmap of DpdkWorkerThread (dpdk_worker_thread.cc:316-342) becomes a
// per-slice 64-bit state word per packet id: high half 0 = not received,
// kRxDone = received in an earlier call, otherwise the claim tag of the frame
// that won it in the current call (larger tag = earlier frame, so a 64-bit
// atomicMax picks the first copy); low byte = that frame's exponent byte, so
// the winner's exponent travels with the claim (PostprocessSingle's
// scaling_factors_[pkt_id], ppp.cc:254-260) and needs no separate pass.
constexpr uint32_t kRxDone = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t rx_tag(uint64_t f) { return 0xFFFFFFFEu - (uint32_t)f; }

struct RxArgs {
    const uint8_t* frames;
    uint64_t nframes;
    uint64_t stride;
    uint64_t numel;
    uint64_t nblocks;           // B
    uint64_t b;                 // extra batch
    unsigned long long* state;  // [B + b]
    int8_t* exps;               // [B]
    float* out;
    unsigned long long* counts; // {accepted, discarded} or nullptr
    uint32_t W;
    uint32_t xcd;           // xcd_block chunk (0 = plain order)
    uint32_t job;               // (uint8_t)job_id
};

// Header dwords 10..12 of frame f: short_job_id = byte 43, pkt_id = bytes
// 44-47 (host order), exponent = byte 50.
struct RxHdr {
    uint32_t pid;
    uint32_t exp;
    bool ok;                    // this job, pkt_id in range
};

typedef uint32_t u3a __attribute__((ext_vector_type(3), aligned(4)));

__device__ __forceinline__ RxHdr rx_header(const RxArgs& a, uint64_t f) {
    // one 12-byte load for dwords 10..12 (the compiler otherwise sinks the
    // dword-12 load behind the job / range check: two round trips).  Default
    // cache policy, not non-temporal: the 128-byte line it fetches also holds
    // the first payload bytes (offset 52), which the apply pass reads next —
    // kept in the caches, that line is not fetched from HBM a second time
    // (cold frame sets: 94.7 -> 91.0 us per 256 MiB rx call,
    // profiles/r05/ab_rx_claim_policy.json).
    const u3a hv = *reinterpret_cast<const u3a*>(a.frames + f * a.stride + 40);
    const uint32_t d10 = hv.x, d11 = hv.y, d12 = hv.z;
    RxHdr r;
    r.pid = d11;
    r.exp = (d12 >> 16) & 0xffu;
    r.ok = (d10 >> 24) == a.job && (uint64_t)d11 < a.nblocks + a.b;
    return r;
}

// Pass 1, thread per frame: frames of another job, out-of-range or already
// received pkt_ids are discarded; the others claim their pkt_id.  Counting:
// accepted = frames - discarded, so block 0 adds the frame count once and only
// workgroups that saw a discard touch the counters (same-address atomics from
// every workgroup serialize in one L2 channel: ~40 us at 262 k frames).
__global__ __launch_bounds__(kBlockThreads) void k_rx_claim(RxArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlockThreads;
    const uint64_t f0 = (uint64_t)blockIdx.x * kBlockThreads + threadIdx.x;
    if (!a.counts) {
        // no counters: non-returning atomics, the wave does not wait for them
        for (uint64_t f = f0; f < a.nframes; f += stride) {
            const RxHdr h = rx_header(a, f);
            if (h.ok) atomicMax(a.state + h.pid, ((unsigned long long)rx_tag(f) << 32) | h.exp);
        }
        return;
    }
    __shared__ uint32_t disc;
    if (threadIdx.x == 0) disc = 0;
    __syncthreads();
    uint32_t mine = 0;
    for (uint64_t f = f0; f < a.nframes; f += stride) {
        const RxHdr h = rx_header(a, f);
        if (!h.ok) { mine++; continue; }
        const unsigned long long v = ((unsigned long long)rx_tag(f) << 32) | h.exp;
        if (atomicMax(a.state + h.pid, v) != 0ull) mine++;          // duplicate or received earlier
    }
    if (mine) atomicAdd(&disc, mine);
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long acc = blockIdx.x == 0 ? (unsigned long long)a.nframes : 0ull;
        acc -= disc;                                                 // mod 2^64
        if (acc) atomicAdd(a.counts + 0, acc);
        if (disc) atomicAdd(a.counts + 1, (unsigned long long)disc);
    }
}

// Pass 2: PostprocessSingle for every winning frame, walked in block order:
// the wave of blocks k .. k + 1024/P - 1 reads state[k + b] (the claim tag of
// the frame that won pkt_id k + b in this call, which names that frame) and
// state[k] (low byte = exponent of block k, held by a winner of this call or
// kRxDone), then gathers the winner's payload and writes out[k*P ..]
// contiguously.  No header is read again; pkt_ids without a winner in this
// call (not received, or received earlier) write nothing; the same pass then
// retires the winners.
// 16-B chunks per lane per tile (slices of 256 elements); a tile holds whole
// packets, so never below P / 256.  2 against 4 on 4 cycled 256 MiB frame
// sets: 97.63 -> 95.59 us per rx call (profiles/r04/ab_rx_slices.json), as
// the plane kernels moved to 2-slice tiles.
__host__ __device__ constexpr int rx_slices(int P) { return P / 256 > 2 ? P / 256 : 2; }

__device__ __forceinline__ bool rx_winner(unsigned long long sw, uint64_t nframes, uint64_t& f) {
    const uint32_t hi = (uint32_t)(sw >> 32);
    f = 0xFFFFFFFEull - hi;                    // rx_tag inverse
    return hi != 0u && hi != kRxDone && f < nframes;
}

template <int P, bool NT = false>
__global__ __launch_bounds__(kBlockThreads) void k_rx_apply(RxArgs a) {
    __shared__ float lut[256];
    // power-of-two W: the table holds exact reciprocals and dequantize multiplies
    // (bit-equal to the IEEE division, rcp_scale_pow2); otherwise scales
    const bool pow2 = (a.W & (a.W - 1)) == 0;
    if (pow2) build_rcp_lut(lut, a.W);
    else build_lut(lut, a.W);
    constexpr int kRxU = rx_slices(P);
    constexpr int kRxTileElems = kRxU * kWave * 4;
    constexpr int kChunksPerFrame = P / 4;     // 16-B chunks per payload
    constexpr int kBlocksPerTile = kRxTileElems / P;
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t ntiles = (a.nblocks + kBlocksPerTile - 1) / kBlocksPerTile;
    for (uint64_t t = xcd_block(a.xcd) * kWavesPerBlock + wave_index(); t < ntiles; t += nwaves) {
        u4a w[kRxU];
        bool ok[kRxU];
        float s[kRxU];
        uint64_t f[kRxU];
        // The state words are read unconditionally (index clamped into the
        // slice) so that all of them are in flight at once: per-slice guarded
        // reads made hipcc wait for each one before issuing the next.
        unsigned long long sw[kRxU], se[kRxU];
        if constexpr (kChunksPerFrame >= kWave) {
            // P >= 256: slice u of the tile lies in one block, so its state
            // words are wave-uniform: scalar loads
            const ConstU64* state = reinterpret_cast<const ConstU64*>(reinterpret_cast<uintptr_t>(a.state));
#pragma unroll
            for (int u = 0; u < kRxU; u++) {
                const uint64_t k = t * kBlocksPerTile + (u * kWave) / kChunksPerFrame;
                const uint64_t kc = k < a.nblocks ? k : a.nblocks - 1;
                sw[u] = state[kc + a.b];
                se[u] = state[kc];
            }
#pragma unroll
            for (int u = 0; u < kRxU; u++) {
                const uint64_t k = t * kBlocksPerTile + (u * kWave) / kChunksPerFrame;
                ok[u] = rx_winner(sw[u], a.nframes, f[u]) && k < a.nblocks;
                s[u] = lut[(uint32_t)se[u] & 0xffu];
            }
        } else {
#pragma unroll
            for (int u = 0; u < kRxU; u++) {
                const uint64_t k = t * kBlocksPerTile + (u * kWave + lane) / kChunksPerFrame;
                const uint64_t kc = k < a.nblocks ? k : a.nblocks - 1;
                sw[u] = a.state[kc + a.b];
                se[u] = a.state[kc];
            }
#pragma unroll
            for (int u = 0; u < kRxU; u++) {
                const uint64_t k = t * kBlocksPerTile + (u * kWave + lane) / kChunksPerFrame;
                ok[u] = rx_winner(sw[u], a.nframes, f[u]) && k < a.nblocks;
                s[u] = lut[(uint32_t)se[u] & 0xffu];
            }
        }
        // Non-temporal payload loads (25 % faster than default-policy loads for
        // this stream, hbm_probe), issued unconditionally so they are all in
        // flight together: a slice without a winner reads frame 0's (L2-hot)
        // bytes instead and its words are zeroed.
#pragma unroll
        for (int u = 0; u < kRxU; u++)
            w[u] = __builtin_nontemporal_load(reinterpret_cast<const u4a*>(
                a.frames + (ok[u] ? f[u] : 0ull) * a.stride + 52 + 16ull * ((u * kWave + lane) % kChunksPerFrame)));
#pragma unroll
        for (int u = 0; u < kRxU; u++)
            if (!ok[u]) w[u] = u4a{0u, 0u, 0u, 0u};
        // Dequantize all slices first, unconditionally (a slice without a
        // winner computes on zeros and is not stored), then store: with the
        // first use of the loaded words inside per-slice conditional blocks,
        // hipcc waited vmcnt(0) — on the previous slice's store too — before
        // every slice.
        f4 o[kRxU];
#pragma unroll
        for (int u = 0; u < kRxU; u++) {
            if (pow2)
                o[u] = mkf4((float)(int32_t)bswap(w[u].x) * s[u], (float)(int32_t)bswap(w[u].y) * s[u],
                            (float)(int32_t)bswap(w[u].z) * s[u], (float)(int32_t)bswap(w[u].w) * s[u]);
            else
                o[u] = mkf4(dequantize1(bswap(w[u].x), s[u]), dequantize1(bswap(w[u].y), s[u]),
                            dequantize1(bswap(w[u].z), s[u]), dequantize1(bswap(w[u].w), s[u]));
        }
#pragma unroll
        for (int u = 0; u < kRxU; u++) {
            if (!ok[u]) continue;
            const uint64_t off = t * kRxTileElems + 4ull * (u * kWave + lane);
            if (off >= a.numel) continue;
            float* p = a.out + off;
            if (a.numel - off >= 4 && ((uintptr_t)p & 15u) == 0) {
                if constexpr (NT) SML_NT_STORE16(o[u], reinterpret_cast<f4*>(p));
                else *reinterpret_cast<f4*>(p) = o[u];
            }
            else store4_guarded(p, o[u], 0, a.numel - off);
        }
        // The commit, folded in (it was a third launch): the lane that owns
        // block k retires this call's winner of pkt_id k + b (state -> kRxDone,
        // exponent byte kept), publishes exps[k] once pkt_id k is received, and
        // for k < b retires the extra-batch pkt_id k too.  Every pkt_id's high
        // half is read and written by exactly one wave (its own); other waves
        // read only the low byte, which the retirement keeps.
#pragma unroll
        for (int u = 0; u < kRxU; u++) {
            const uint64_t k = t * kBlocksPerTile + (u * kWave + lane) / kChunksPerFrame;
            if (((u * kWave + lane) % kChunksPerFrame) != 0 || k >= a.nblocks) continue;
            const uint32_t hw = (uint32_t)(sw[u] >> 32), he = (uint32_t)(se[u] >> 32);
            if (hw != 0u && hw != kRxDone)
                a.state[k + a.b] = ((unsigned long long)kRxDone << 32) | (sw[u] & 0xffull);
            if (he != 0u) a.exps[k] = (int8_t)(se[u] & 0xffull);
            if (k < a.b && he != 0u && he != kRxDone)
                a.state[k] = ((unsigned long long)kRxDone << 32) | (se[u] & 0xffull);
        }
    }
}

// --------------------------------------- INT32 job slices, receive side
//
// An INT32 frame is self-contained — pkt_id k carries block k's words and
// there is no exponent to take from another frame (NeedsExtraBatch false,
// ppp.cc:65-67; PostprocessSingle's INT32 branch, ppp.cc:262-298) — so one
// pass in stream order decides and writes each frame: no claim pass over the
// headers, no second walk in block order.  State: uint64[2B + 6] per slice:
// [0, B) the rx bitmap, [B] the call sequence c of this slice, [B + 1] the
// conflicts resolved in the slice so far (a statistic: copies that arrived
// ahead of an earlier one), [B + 2 + (c & 1)] the conflict count of call c,
// [B + 4 + (c & 1)] the length of call c's dirty list, [B + 6, 2B + 6) that
// list: the pkt_ids marked dirty in call c (appended by the claim that sets
// a pkt_id's dirty bit), so the fix-up visits only them.  The per-call
// counters alternate between two slots so that the fix-up's workgroups can
// all read call c's without a grid-wide barrier: the fix-up of call c clears
// the OTHER slot (call c - 1's, whose fix-up has ended), ready for c + 1.
// A frame's tag is
//   (0xFFFFFFFF - c) << 32 | (0x7FFFFFFF - f) << 1      (bit 0: dirty),
// larger for an earlier call and, within a call, for an earlier frame f, so
// a 64-bit atomicMax on state[pkt_id] keeps the first copy of the stream,
// and a pkt_id accepted by an earlier call (higher tag) discards every later
// copy — the reference's "seen before" test (dpdk_worker_thread.cc:316-342)
// without a retirement pass.  The atomic's old value decides:
//   0                  first claim of the pkt_id: write, accepted;
//   above the tag      an earlier copy (or call) holds it: discarded;
//   below the tag      this frame is earlier than the copy that claimed first
//                      and already wrote: write too, mark the pkt_id dirty,
//                      count a conflict (the counts stay exact: the displaced
//                      copy was counted accepted, this one is counted as the
//                      discard).
// Which of two racing writes lands last is not ordered, so the fix-up
// (k_rx_int32_fixup, same stream) rewrites every dirty pkt_id from its final
// winner — the highest tag, the first copy — and then advances c.  It walks
// the dirty list over a grid of workgroups (not one workgroup
// scanning all B state words for one conflict); a list that overflowed its
// B entries (one pkt_id can be appended again when a later claim's
// atomicMax clears its dirty bit for an instant) falls back to the scan of
// every state word, over the same grid.  Copies
// of one pkt_id are normally identical (retransmissions), but the rule holds
// for any payloads.
constexpr uint32_t kRxI32MaxFrames = 0x7FFFFFFFu;
constexpr uint32_t kRxFixupBlocks = 128;   // k_rx_int32_fixup's grid

__host__ __device__ constexpr int rx_int32_slices(int P) { return P / 256 > 4 ? P / 256 : 4; }

__device__ __forceinline__ unsigned long long rx_int32_tag(uint32_t call, uint64_t f) {
    return ((unsigned long long)(0xFFFFFFFFu - call) << 32) | ((unsigned long long)(kRxI32MaxFrames - (uint32_t)f) << 1);
}

// A wave takes F = U * 256 / P consecutive frames per tile (4 frames at
// P = 256): every lane loads one of the tile's F headers (lane l < F's is
// the one used) and its 16-byte payload chunks; lane l < F then makes frame
// l's claim, and the decision and the pkt_id are shuffled to the lanes
// holding that frame's chunks.  Software-pipelined: the next tile's header
// and payload loads are issued before this tile's claim, so a wave waits on
// one round trip per tile (the claim's, with the next loads under it) rather
// than two in series (loads, then the claim).
template <int P>
struct RxI32Tile {
    static constexpr int kU = rx_int32_slices(P);
    u3a hv;
    u4a w[kU];
};

template <int P>
__device__ __forceinline__ void rx_int32_load(const RxArgs& a, uint64_t t, int lane, RxI32Tile<P>& r) {
    constexpr int kU = RxI32Tile<P>::kU;
    constexpr int kChunksPerFrame = P / 4;
    constexpr int kF = kU * kWave / kChunksPerFrame;
    const uint64_t f0 = t * kF;
    // header first (the claim needs it first); indices clamped into the call
    // so every load is unconditional and in flight at once
    uint64_t fh = f0 + (uint64_t)(lane % kF);
    fh = fh < a.nframes ? fh : a.nframes - 1;
    r.hv = *reinterpret_cast<const u3a*>(a.frames + fh * a.stride + 40);
#pragma unroll
    for (int u = 0; u < kU; u++) {
        const int c = u * kWave + lane;
        uint64_t f = f0 + c / kChunksPerFrame;
        f = f < a.nframes ? f : a.nframes - 1;
        r.w[u] = __builtin_nontemporal_load(reinterpret_cast<const u4a*>(
            a.frames + f * a.stride + 52 + 16ull * (c % kChunksPerFrame)));
    }
}

template <int P, bool NT>
__global__ __launch_bounds__(kBlockThreads) void k_rx_int32(RxArgs a) {
    constexpr int kU = RxI32Tile<P>::kU;
    constexpr int kChunksPerFrame = P / 4;
    constexpr int kF = kU * kWave / kChunksPerFrame;          // frames per tile
    static_assert(kF >= 1 && kF <= kWave, "frames per tile");
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t ntiles = (a.nframes + kF - 1) / kF;
    const uint32_t call = (uint32_t)a.state[a.nblocks];
    unsigned long long* const conflicts = a.state + a.nblocks + 2 + (call & 1u);
    unsigned long long* const listed = a.state + a.nblocks + 4 + (call & 1u);
    uint32_t disc = 0;
    uint64_t t = xcd_block(a.xcd) * kWavesPerBlock + wave_index();
    RxI32Tile<P> cur, nxt;
    if (t < ntiles) rx_int32_load<P>(a, t, lane, cur);
    for (; t < ntiles; t += nwaves) {
        const uint64_t tn = t + nwaves;
        if (tn < ntiles) rx_int32_load<P>(a, tn, lane, nxt);
        const uint64_t f0 = t * kF;
        // lane l < kF: the claim of frame f0 + l
        bool write = false;
        uint32_t pid = cur.hv.y;
        if (lane < kF && f0 + lane < a.nframes) {
            const uint64_t f = f0 + lane;
            const bool ok = (cur.hv.x >> 24) == a.job && (uint64_t)pid < a.nblocks;
            bool keep = false;
            if (ok) {
                const unsigned long long tag = rx_int32_tag(call, f);
                const unsigned long long old = atomicMax(a.state + pid, tag);
                if (old == 0ull) {
                    write = true;
                    keep = true;
                } else if ((old & ~1ull) < tag) {
                    write = true;
                    atomicAdd(conflicts, 1ull);
                    if (!(atomicOr(a.state + pid, 1ull) & 1ull)) {   // this claim made it dirty: list it
                        const unsigned long long i = atomicAdd(listed, 1ull);
                        if (i < a.nblocks) a.state[a.nblocks + 6 + i] = pid;
                    }
                }
            }
            if (!keep) disc++;
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int c = u * kWave + lane;
            const int src = c / kChunksPerFrame;
            const bool wr = __shfl(write ? 1 : 0, src) != 0;
            const uint64_t k = (uint32_t)__shfl((int)pid, src);
            if (!wr) continue;
            const uint64_t off = k * P + 4ull * (c % kChunksPerFrame);
            if (off >= a.numel) continue;
            const u4a& w = cur.w[u];
            const f4 o = __builtin_bit_cast(f4, mku4(bswap(w.x), bswap(w.y), bswap(w.z), bswap(w.w)));
            float* p = a.out + off;
            if (a.numel - off >= 4 && ((uintptr_t)p & 15u) == 0) {
                // a wave's F frames land anywhere in the output (their pkt_ids),
                // so not SML_NT_STORE16: its buffer resource spans +-1 GiB
                // around the first lane's address
                if constexpr (NT) SML_NT_STORE16_UNALIGNED(o, reinterpret_cast<f4*>(p));
                else *reinterpret_cast<f4*>(p) = o;
            }
            else store4_guarded(p, o, 0, a.numel - off);
        }
        cur = nxt;
    }
    if (!a.counts) return;
    // accepted = frames - discarded: block 0 adds the frame count once, and
    // only workgroups that saw a discard touch the discard counter
    __shared__ uint32_t bdisc;
    if (threadIdx.x == 0) bdisc = 0;
    __syncthreads();
    if (disc) atomicAdd(&bdisc, disc);
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long acc = blockIdx.x == 0 ? (unsigned long long)a.nframes : 0ull;
        acc -= bdisc;                                                // mod 2^64
        if (acc) atomicAdd(a.counts + 0, acc);
        if (bdisc) atomicAdd(a.counts + 1, (unsigned long long)bdisc);
    }
}

// Rewrite dirty pkt_id k from the frame its tag names (the first copy), the
// whole wave lane-strided over the block's words.
__device__ __forceinline__ void rx_int32_rewrite(const RxArgs& a, uint32_t P, uint64_t k, unsigned long long s,
                                                 int lane) {
    const uint64_t f = kRxI32MaxFrames - ((uint32_t)s >> 1);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.frames + f * a.stride + 52);
    uint32_t* dst = reinterpret_cast<uint32_t*>(a.out) + k * P;
    const uint64_t valid = a.numel - k * P < P ? a.numel - k * P : P;
    for (uint64_t i = lane; i < valid; i += kWave) dst[i] = bswap(src[i]);
}

// kRxFixupBlocks workgroups, after k_rx_int32 on the same stream: with
// conflicts in this call, every dirty pkt_id is rewritten from the frame its
// tag names (the first copy) and cleaned; the slice's conflict total
// accumulates, the other counter slot is cleared and the call sequence
// advanced.  Without conflicts (no copies claimed out of order) it only does
// the last three.
__global__ __launch_bounds__(kBlockThreads) void k_rx_int32_fixup(RxArgs a, uint32_t P) {
    const unsigned long long call = a.state[a.nblocks];
    const uint32_t slot = (uint32_t)call & 1u;
    const unsigned long long n = a.state[a.nblocks + 2 + slot];
    const unsigned long long listed = a.state[a.nblocks + 4 + slot];
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + wave_index();
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    if (n && listed <= a.nblocks) {
        // the dirty list, one pkt_id per wave at a time; the wave that finds
        // the bit set rewrites the block, then cleans the bit (an id listed
        // twice is rewritten twice with the same words, or found clean)
        for (uint64_t i = wave; i < listed; i += nwaves) {
            const uint64_t k = a.state[a.nblocks + 6 + i];
            const unsigned long long s = a.state[k];
            if (s & 1ull) {
                rx_int32_rewrite(a, P, k, s, lane);
                if (lane == 0) a.state[k] = s & ~1ull;
            }
        }
    } else if (n) {
        // the list overflowed: every state word, 64 per wave at a time; the
        // dirty ones (a ballot) rewritten one after another by the whole wave
        for (uint64_t k0 = wave * kWave; k0 < a.nblocks; k0 += nwaves * kWave) {
            const uint64_t k = k0 + lane;
            const unsigned long long s = k < a.nblocks ? a.state[k] : 0ull;
            unsigned long long dirty = __ballot((s & 1ull) != 0);
            while (dirty) {
                const int j = __builtin_ctzll(dirty);
                dirty &= dirty - 1;
                const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)s, j);
                rx_int32_rewrite(a, P, k0 + j, lo, lane);
            }
            if (s & 1ull) a.state[k] = s & ~1ull;
        }
    }
    // one thread of the grid: the slice's total, the other slot cleared (call
    // c - 1's: its fix-up has ended) for call c + 1, the sequence advanced.
    // No workgroup of this launch reads those words after its start, and the
    // next rx call runs after the whole launch (stream order).
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (n) a.state[a.nblocks + 1] += n;
        a.state[a.nblocks + 2 + (slot ^ 1u)] = 0ull;
        a.state[a.nblocks + 4 + (slot ^ 1u)] = 0ull;
        a.state[a.nblocks] = call + 1;
    }
}

// ------------------------------------------------------------ host side

template <bool ALIGNED, bool GLOBAL, bool I32 = false>
static void launch_frames_p(uint32_t P, bool nts, dim3 grid, hipStream_t st, const FrameArgs& a) {
#define SML_FR(PN)                                                                                   \
    if (nts) k_quantize_frames<PN, ALIGNED, GLOBAL, true, I32><<<grid, kBlockThreads, 0, st>>>(a);   \
    else k_quantize_frames<PN, ALIGNED, GLOBAL, false, I32><<<grid, kBlockThreads, 0, st>>>(a);
    switch (P) {
        case 64:   SML_FR(64) break;
        case 128:  SML_FR(128) break;
        case 256:  SML_FR(256) break;
        case 512:  SML_FR(512) break;
        default:   SML_FR(1024) break;
    }
#undef SML_FR
}

template <bool NT>
static void launch_rx_apply_nt(uint32_t P, dim3 grid, hipStream_t st, const RxArgs& a) {
    switch (P) {
        case 64:   k_rx_apply<64, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 128:  k_rx_apply<128, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 256:  k_rx_apply<256, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 512:  k_rx_apply<512, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
        default:   k_rx_apply<1024, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
    }
}

// The output of a slice from the non-temporal threshold on takes
// non-temporal stores, as K4's does (sml_set_payload_nt_threshold).
static void launch_rx_apply(uint32_t P, dim3 grid, hipStream_t st, const RxArgs& a) {
    if (4 * a.numel >= g_nt_threshold.load(std::memory_order_relaxed)) launch_rx_apply_nt<true>(P, grid, st, a);
    else launch_rx_apply_nt<false>(P, grid, st, a);
}

template <bool NT>
static void launch_rx_int32_nt(uint32_t P, dim3 grid, hipStream_t st, const RxArgs& a) {
    switch (P) {
        case 64:   k_rx_int32<64, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 128:  k_rx_int32<128, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 256:  k_rx_int32<256, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
        case 512:  k_rx_int32<512, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
        default:   k_rx_int32<1024, NT><<<grid, kBlockThreads, 0, st>>>(a); break;
    }
}

}  // namespace sml

using namespace sml;

extern "C" {

uint64_t sml_frame_bytes(uint32_t packet_numel) { return 52ull + 4ull * packet_numel; }

uint64_t sml_rx_state_words(uint64_t numel, uint32_t packet_numel, uint32_t batch_max, int int32) {
    if (!valid_packet(packet_numel)) return 0;
    const uint64_t B = sml_num_blocks(numel, packet_numel);
    if (int32) return 2 * B + 6;   // bitmap, sequence, conflict counts, dirty list (k_rx_int32)
    const uint64_t w = B + (B < batch_max ? B : batch_max);
    return w ? w : 1;
}

}  // extern "C"

namespace sml {

// FrameArgs of one slice's frames: geometry, pool indices and the constant
// header bytes 0..43 (BuildPacket, dpdk_worker_thread_utils.inc:76-126).
static void frame_args(const sml_frame_params* prm, uint64_t numel, uint32_t P, uint16_t W, uint64_t b,
                       void* frames, uint64_t stride, FrameArgs& a) {
    a.xcd = g_xcd_chunk.load(std::memory_order_relaxed);
    a.numel = numel;
    a.nblocks = sml_num_blocks(numel, P);
    a.ntiles = (a.nblocks * P + kTileElems - 1) / kTileElems;
    a.b = b;
    a.gexp = nullptr;
    a.frames = static_cast<uint8_t*>(frames);
    a.stride = stride;
    a.W = W;
    a.pool_start = prm->pool_index_start;
    a.pool_shift = prm->pool_index_shift;
    a.mop = prm->max_outstanding_pkts ? prm->max_outstanding_pkts : 1;
    uint8_t h[44];
    memset(h, 0, sizeof(h));
    const uint32_t data_len = (uint32_t)sml_frame_bytes(P);
    memcpy(h + 0, prm->dst_mac, 6);
    memcpy(h + 6, prm->src_mac, 6);
    h[12] = 0x08; h[13] = 0x00;                              // RTE_ETHER_TYPE_IPV4
    h[14] = 0x45;                                            // version_ihl
    h[16] = (uint8_t)((data_len - 14) >> 8); h[17] = (uint8_t)(data_len - 14);
    h[22] = 128;                                             // time_to_live
    h[23] = 17;                                              // IPPROTO_UDP
    memcpy(h + 26, &prm->src_ip_be, 4);
    memcpy(h + 30, &prm->dst_ip_be, 4);
    memcpy(h + 34, &prm->src_port_be, 2);
    memcpy(h + 36, &prm->dst_port_be, 2);
    h[38] = (uint8_t)((data_len - 34) >> 8); h[39] = (uint8_t)(data_len - 34);
    // udp->dgram_cksum = rte_ipv4_phdr_cksum(ip, ol_flags): raw 16-bit sum of the pseudo header
    uint8_t psd[12] = {h[26], h[27], h[28], h[29], h[30], h[31], h[32], h[33], 0, 17,
                       (uint8_t)((data_len - 34) >> 8), (uint8_t)(data_len - 34)};
    uint32_t sum = 0;
    for (int i = 0; i < 12; i += 2) sum += (uint32_t)psd[i] | ((uint32_t)psd[i + 1] << 8);
    sum = (sum & 0xffff) + (sum >> 16);
    sum = (sum & 0xffff) + (sum >> 16);
    h[40] = (uint8_t)sum; h[41] = (uint8_t)(sum >> 8);
    h[42] = (uint8_t)((1 << 4) + (P < 64 ? 0 : P < 128 ? 1 : P < 256 ? 2 : 3));  // job_type_size
    h[43] = (uint8_t)prm->job_id;                                                // short_job_id
    memcpy(a.hdr, h, 44);
}

// Payload store policy: non-temporal for a frame set in device memory from
// the threshold on (written once, handed on); host frames (a NIC's pinned
// mbufs) keep the default policy.
static bool frames_nt(const void* frames, uint64_t bytes) {
    if (bytes < g_nt_threshold.load(std::memory_order_relaxed)) return false;
    hipPointerAttribute_t pa;
    if (hipPointerGetAttributes(&pa, frames) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return pa.type == hipMemoryTypeDevice;
}

}  // namespace sml

extern "C" {

sml_status_t sml_quantize_pack_frames(const float* d_in, uint64_t numel, uint32_t P, uint16_t W,
                                      const int8_t* d_global_exps, uint32_t batch_max,
                                      const sml_frame_params* prm, void* frames, uint64_t stride, void* stream) {
    if (!valid_packet(P)) return SML_ERR_UNSUPPORTED;
    if (W == 0 || !prm || batch_max == 0) return SML_ERR_INVALID_ARG;
    if (numel == 0) return SML_OK;
    if (!d_in || !aligned4(d_in) || !frames) return SML_ERR_INVALID_ARG;
    if (!aligned4(frames) || stride % 4 || stride < sml_frame_bytes(P)) return SML_ERR_ALIGNMENT;
    FrameArgs a;
    const uint64_t B = sml_num_blocks(numel, P);
    frame_args(prm, numel, P, W, B < batch_max ? B : batch_max, frames, stride, a);
    a.in = d_in;
    a.gexp = d_global_exps;
    dim3 grid(grid_for_tiles(a.ntiles));
    hipStream_t st = (hipStream_t)stream;
    const bool al = aligned16(d_in);
    const bool nts = frames_nt(frames, (a.nblocks + a.b) * stride);
    if (d_global_exps) { if (al) launch_frames_p<true, true>(P, nts, grid, st, a); else launch_frames_p<false, true>(P, nts, grid, st, a); }
    else               { if (al) launch_frames_p<true, false>(P, nts, grid, st, a); else launch_frames_p<false, false>(P, nts, grid, st, a); }
    return launch_check();
}

sml_status_t sml_pack_frames_int32(const int32_t* d_in, uint64_t numel, uint32_t P, const sml_frame_params* prm,
                                   void* frames, uint64_t stride, void* stream) {
    if (!valid_packet(P)) return SML_ERR_UNSUPPORTED;
    if (!prm) return SML_ERR_INVALID_ARG;
    if (numel == 0) return SML_OK;
    if (!d_in || !aligned4(d_in) || !frames) return SML_ERR_INVALID_ARG;
    if (!aligned4(frames) || stride % 4 || stride < sml_frame_bytes(P)) return SML_ERR_ALIGNMENT;
    FrameArgs a;
    frame_args(prm, numel, P, 1, 0, frames, stride, a);       // INT32: no extra batch
    a.in = reinterpret_cast<const float*>(d_in);              // words moved as bits
    dim3 grid(grid_for_tiles(a.ntiles));
    hipStream_t st = (hipStream_t)stream;
    const bool nts = frames_nt(frames, a.nblocks * stride);
    if (aligned16(d_in)) launch_frames_p<true, false, true>(P, nts, grid, st, a);
    else launch_frames_p<false, false, true>(P, nts, grid, st, a);
    return launch_check();
}

sml_status_t sml_dequantize_frames(const void* frames, uint64_t num_frames, uint64_t stride,
                                   uint64_t numel, uint32_t P, uint16_t W, uint32_t batch_max,
                                   uint64_t job_id, int8_t* d_exps, uint64_t* d_state, float* d_out,
                                   uint64_t* d_counts, void* stream) {
    if (!valid_packet(P)) return SML_ERR_UNSUPPORTED;
    if (W == 0 || batch_max == 0) return SML_ERR_INVALID_ARG;
    if (num_frames == 0) return SML_OK;
    if (num_frames >= 0xFFFFFFFEull) return SML_ERR_UNSUPPORTED;
    if (!frames || !d_state || (numel && (!d_exps || !d_out))) return SML_ERR_INVALID_ARG;
    if (!aligned4(frames) || !aligned4(d_out) || stride % 4 || stride < sml_frame_bytes(P)) return SML_ERR_ALIGNMENT;
    if (((uintptr_t)d_state & 7u) || (d_counts && ((uintptr_t)d_counts & 7u))) return SML_ERR_ALIGNMENT;
    RxArgs a;
    const uint32_t U = (uint32_t)rx_slices((int)P);
    a.xcd = U < 4 ? g_xcd_chunk.load(std::memory_order_relaxed) * (4 / U)   // XCD runs keep their byte length
                  : g_xcd_chunk.load(std::memory_order_relaxed);
    a.frames = static_cast<const uint8_t*>(frames);
    a.nframes = num_frames;
    a.stride = stride;
    a.numel = numel;
    a.nblocks = sml_num_blocks(numel, P);
    a.b = a.nblocks < batch_max ? a.nblocks : batch_max;
    a.state = reinterpret_cast<unsigned long long*>(d_state);
    a.exps = d_exps;
    a.out = d_out;
    a.counts = reinterpret_cast<unsigned long long*>(d_counts);
    a.W = W;
    a.job = (uint8_t)job_id;
    hipStream_t st = (hipStream_t)stream;
    k_rx_claim<<<grid_for_vec(num_frames), kBlockThreads, 0, st>>>(a);
    const uint64_t tile = (uint64_t)U * kWave * 4;
    const uint64_t ntiles = (a.nblocks * P + tile - 1) / tile;
    if (ntiles) launch_rx_apply(P, dim3(grid_for_tiles(ntiles)), st, a);
    return launch_check();
}

sml_status_t sml_unpack_frames_int32(const void* frames, uint64_t num_frames, uint64_t stride, uint64_t numel,
                                     uint32_t P, uint64_t job_id, uint64_t* d_state, int32_t* d_out,
                                     uint64_t* d_counts, void* stream) {
    if (!valid_packet(P)) return SML_ERR_UNSUPPORTED;
    if (num_frames == 0) return SML_OK;
    if (num_frames > kRxI32MaxFrames) return SML_ERR_UNSUPPORTED;
    if (!frames || !d_state || (numel && !d_out)) return SML_ERR_INVALID_ARG;
    if (!aligned4(frames) || !aligned4(d_out) || stride % 4 || stride < sml_frame_bytes(P)) return SML_ERR_ALIGNMENT;
    if (((uintptr_t)d_state & 7u) || (d_counts && ((uintptr_t)d_counts & 7u))) return SML_ERR_ALIGNMENT;
    RxArgs a;
    a.xcd = g_xcd_chunk.load(std::memory_order_relaxed);
    a.frames = static_cast<const uint8_t*>(frames);
    a.nframes = num_frames;
    a.stride = stride;
    a.numel = numel;
    a.nblocks = sml_num_blocks(numel, P);
    a.b = 0;                                                  // INT32: no extra batch
    a.state = reinterpret_cast<unsigned long long*>(d_state);
    a.exps = nullptr;
    a.out = reinterpret_cast<float*>(d_out);                  // words stored as bits
    a.counts = reinterpret_cast<unsigned long long*>(d_counts);
    a.W = 1;
    a.job = (uint8_t)job_id;
    hipStream_t st = (hipStream_t)stream;
    const uint64_t frames_per_tile = (uint64_t)rx_int32_slices((int)P) * kWave * 4 / P;
    const dim3 grid(grid_for_tiles((num_frames + frames_per_tile - 1) / frames_per_tile));
    if (4 * numel >= g_nt_threshold.load(std::memory_order_relaxed)) launch_rx_int32_nt<true>(P, grid, st, a);
    else launch_rx_int32_nt<false>(P, grid, st, a);
    // a grid that spreads a call's dirty pkt_ids over the chip; with no
    // conflict its workgroups read two words and end
    k_rx_int32_fixup<<<kRxFixupBlocks, kBlockThreads, 0, st>>>(a, P);
    return launch_check();
}

sml_status_t sml_rx_reset(uint64_t* d_state, uint64_t num_words, void* stream) {
    if (num_words == 0) return SML_OK;
    if (!d_state || ((uintptr_t)d_state & 7u)) return SML_ERR_INVALID_ARG;
    return hip_check(hipMemsetAsync(d_state, 0, num_words * 8, (hipStream_t)stream));
}

}  // extern "C"
