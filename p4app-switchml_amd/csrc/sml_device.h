// sml_device.h — device-side building blocks shared by the gfx950 kernels of
// SwitchML's end-host pre/post-processor (sml_quantizer.hip: planes;
// sml_frames.hip: DPDK frames).
//
// What the reference does per 1 KiB LTU on one CPU thread
// (client_lib/src/prepostprocessors/cpu_exponent_quantizer_ppp.cc, "ppp.cc"),
// these kernels do for a whole job slice per launch.  The work is a pure
// HBM stream (8 B/element for quantize+pack), so the design rules are the
// streaming ones: 16-B-per-lane coalesced loads/stores (1 KiB per wave
// instruction), several loads in flight per lane, the per-packet max-|x|
// reduce in registers + cross-lane (DPP row ops + v_readlane), no LDS
// round trip for the data, no MFMA (nothing here is a contraction).
//
// Work unit: a "tile" = 1024 consecutive elements of the slice = 4 x f4
// per lane of one wave64.  Slice u of a tile (u = 0..3) is 256 consecutive
// elements, lane l holds elements [u*256 + 4l, u*256 + 4l + 4).  A packet of
// P elements therefore spans P/4 lanes of one slice (P <= 256) or P/256
// whole slices (P = 512, 1024); every packet lies inside one tile.
//
// Arithmetic parity with the VCL=0 reference build:
//  * exponent: integer max of (bits & 0x7fffffff) with NaN bit patterns
//    mapped to 0 == the float '>' scan from 0 at ppp.cc:141-146; then
//    ((m >> 23) & 0xff) - 126 truncated to int8 (ppp.cc:154).
//  * scale: (float)(double(INT32_MAX) / ((float)W * 2^e)) (ppp.cc:257-258),
//    computed once per workgroup into an LDS table.
//  * quantize: roundf(x * s) half away from zero, then the x86-64
//    cvttss2si-to-64-bit-then-truncate conversion (NaN/inf/|r| >= 2^63 -> 0,
//    2^31 <= |r| < 2^63 wraps mod 2^32), then bswap (htonl) — ppp.cc:103.
//  * dequantize: (float)(int32)ntohl(q) / s with IEEE division (ppp.cc:240-241).
//  * f32 denormals are preserved (the kernels are built without
//    -fgpu-flush-denormals-to-zero and without fast-math).
#ifndef SML_DEVICE_H_
#define SML_DEVICE_H_

#include <hip/hip_runtime.h>

#include <stdint.h>

namespace sml {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));
// 16-byte vector with 4-byte alignment: gfx950 runs in unaligned-access mode,
// so this is still one global_store_dwordx4 (used at the 52-byte frame offset).
typedef uint32_t u4a __attribute__((ext_vector_type(4), aligned(4)));
typedef float f4a __attribute__((ext_vector_type(4), aligned(4)));
// Read-only views through the scalar data cache (s_load) for wave-uniform
// metadata (exponent bytes, frame headers, rx state); loads only — nothing in
// these kernels writes through the scalar cache.
typedef const uint32_t __attribute__((address_space(4))) ConstU32;
typedef const unsigned long long __attribute__((address_space(4))) ConstU64;

__device__ __forceinline__ f4 mkf4(float a, float b, float c, float d) { return f4{a, b, c, d}; }
__device__ __forceinline__ u4 mku4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return u4{a, b, c, d}; }

constexpr int kWave = 64;
constexpr int kBlockThreads = 256;
constexpr int kWavesPerBlock = kBlockThreads / kWave;
constexpr int kU = 4;                          // f4 slices per lane per tile
constexpr int kTileElems = kWave * 4 * kU;     // 1024
// Elements of a tile of U slices (K1/K2/K3 take U = 1, 2 or 4: DESIGN §4).
template <int U>
constexpr int tile_elems() { return kWave * 4 * U; }

// ----------------------------------------------------------------- numerics

// ppp.cc:257-258.  powf(2, e) is exactly 2^e for every int8 e (2^-127 and
// 2^-128 are denormal but exact), so ldexp gives the same float; the product
// with (float)W is a float multiply (overflow -> inf -> scale 0, as on x86);
// the quotient is a correctly rounded double division, rounded to float.
__device__ __forceinline__ float scale_of(uint32_t W, int e) {
    float denom = (float)W * __builtin_ldexpf(1.0f, e);
    return (float)(2147483647.0 / (double)denom);
}

// |x| bits with NaN mapped to 0: a NaN never wins the reference's '>' scan.
__device__ __forceinline__ uint32_t absbits(float x) {
    uint32_t a = __float_as_uint(x) & 0x7fffffffu;
    return a > 0x7f800000u ? 0u : a;
}

__device__ __forceinline__ int exponent_of(uint32_t maxbits) {
    // ppp.cc:154 computes in int and stores through int8_t*: 129 -> -127, 128 -> -128.
    return (int)(int8_t)(uint8_t)(((maxbits >> 23) & 0xffu) - 126u);
}

// gcc/x86-64 lowering of the float -> uint32 conversion at ppp.cc:103:
// cvttss2si into a 64-bit register, low 32 bits kept.  Needed only for
// |r| >= 2^31 or NaN (r is already integral); below that it equals v_cvt_i32_f32.
__device__ __forceinline__ uint32_t x86_wrap(float r) {
    uint32_t b = __float_as_uint(r);
    uint32_t E = (b >> 23) & 0xffu;
    if (E >= 190u) return 0u;                  // |r| >= 2^63, inf, NaN -> 0x8000...0 -> low 0
    uint32_t m = (b & 0x7fffffu) | 0x800000u;
    uint32_t sh = E - 150u;                    // >= 8 here
    uint32_t low = sh < 32u ? (m << sh) : 0u;
    return (b >> 31) ? (0u - low) : low;
}

// Quantize 4 consecutive elements with one scale (host byte order result).
// RNE_BODY: lanes [0, body) use the VCL=1 roundi() semantics (RNE, out of
// range / NaN -> 0x80000000); the rest use the VCL=0 scalar path.  With
// RNE == false every element takes the scalar path.
template <bool RNE>
__device__ __forceinline__ u4 quantize4(f4 x, float s, uint64_t idx, uint64_t body) {
    const float p[4] = {x.x * s, x.y * s, x.z * s, x.w * s};
    uint32_t q[4];
    bool wide = false;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if (RNE && idx + j < body) {
            q[j] = fabsf(p[j]) < 0x1p31f ? (uint32_t)(int32_t)__builtin_rintf(p[j]) : 0x80000000u;
        } else {
            float r = __builtin_roundf(p[j]);      // half away from zero, like std::round(float)
            q[j] = (uint32_t)(int32_t)r;           // exact whenever |r| < 2^31
            wide |= !(fabsf(r) < 0x1p31f);
        }
    }
    if (__builtin_expect(wide, 0)) {               // rare: out-of-range / NaN / inf products
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (RNE && idx + j < body) continue;
            float r = __builtin_roundf(p[j]);
            if (!(fabsf(r) < 0x1p31f)) q[j] = x86_wrap(r);
        }
    }
    return mku4(q[0], q[1], q[2], q[3]);
}

__device__ __forceinline__ float dequantize1(uint32_t q_host_order, float s) {
    return (float)(int32_t)q_host_order / s;
}

__device__ __forceinline__ uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }

// ------------------------------------------------------------- memory ops

// ALIGNED = false: slices that start at any 4-byte offset (FIFO slices,
// fifo_scheduler.cc:93-109).  gfx950 runs in unaligned mode and moves 4-byte
// aligned 16-B accesses at the full stream rate (hbm_probe: +4 B offset
// loads 7.15 TB/s, stores 7.20 TB/s vs 7.23 aligned), so both forms are one
// dwordx4 per lane.
template <bool ALIGNED>
__device__ __forceinline__ f4 load4(const float* p) {
    if constexpr (ALIGNED) {
        return __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
    } else {
        const f4a v = __builtin_nontemporal_load(reinterpret_cast<const f4a*>(p));
        return mkf4(v.x, v.y, v.z, v.w);
    }
}

__device__ __forceinline__ f4 load4_guarded(const float* p, uint64_t idx, uint64_t numel) {
    f4 v;
    v.x = idx + 0 < numel ? p[0] : 0.0f;
    v.y = idx + 1 < numel ? p[1] : 0.0f;
    v.z = idx + 2 < numel ? p[2] : 0.0f;
    v.w = idx + 3 < numel ? p[3] : 0.0f;
    return v;
}

// The non-temporal 16-byte store of every streaming kernel's large-output
// path (planes and fp32 outputs from g_nt_threshold on, 16-byte aligned):
// `sc1 nt` (device coherence scope, streaming).  On cold buckets against the
// `nt` of __builtin_nontemporal_store: K1 -1.2 %, K4 -2.8 %, the round trip
// -0.9 % at 256 MiB, K4 -3.2 % at 128 MiB (profiles/r04/ab_bufpol.json).
// No builtin sets these bits on a global store, so it is a buffer store the
// compiler schedules (hazards, waits): a descriptor based 1 GiB below the
// first active lane's address — every lane of a wave stores within a few KiB
// of it — and the lane's byte offset from that base.  Never inline asm: the
// hazard recognizer cannot see into it.
// The first active lane's 64-bit value, in SGPRs.  readfirstlane returns a
// signed int: each half goes through uint32_t before it is widened (a sign-
// extended low half corrupts the high one).
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
template <typename V>
__device__ __forceinline__ void nt_store16_sc1(V v, void* p) {
    static_assert(sizeof(V) == 16, "16-byte stores only");
    typedef uint32_t w4 __attribute__((ext_vector_type(4)));
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint64_t base = uniform_u64(a) - (1ull << 30);
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(w4, v), r, (int)(uint32_t)(a - base), 0,
                                           18 /* sc1 nt */);
}
#define SML_NT_STORE16(v, p) nt_store16_sc1((v), (void*)(p))
#define SML_NT_STORE16_UNALIGNED(v, p) __builtin_nontemporal_store((v), (p))

// NT: non-temporal (for output planes larger than the Infinity Cache: see
// g_nt_threshold in sml_quantizer.hip); default policy otherwise.
template <bool ALIGNED, bool NT = false>
__device__ __forceinline__ void store4(float* p, f4 v) {
    if constexpr (ALIGNED) {
        if constexpr (NT) SML_NT_STORE16(v, reinterpret_cast<f4*>(p));
        else *reinterpret_cast<f4*>(p) = v;   // default policy: faster than nt stores up to 256 MiB
    } else {
        if constexpr (NT) SML_NT_STORE16_UNALIGNED((f4a{v.x, v.y, v.z, v.w}), reinterpret_cast<f4a*>(p));
        else *reinterpret_cast<f4a*>(p) = f4a{v.x, v.y, v.z, v.w};
    }
}

__device__ __forceinline__ void store4_guarded(float* p, f4 v, uint64_t idx, uint64_t numel) {
    if (idx + 0 < numel) p[0] = v.x;
    if (idx + 1 < numel) p[1] = v.y;
    if (idx + 2 < numel) p[2] = v.z;
    if (idx + 3 < numel) p[3] = v.w;
}

// Payload stores keep the default cache policy: measured 9 % faster than
// non-temporal stores on the 256 MiB bucket (loads stay non-temporal,
// which is 15 % faster than default-policy loads) — profiles/r01/ab*.json.
__device__ __forceinline__ void store_payload(u4* dst, u4 q) { *dst = q; }
// Past the Infinity Cache's reach (a slice whose payload plane cannot stay
// resident) non-temporal payload stores stream faster: K1 picks the policy by
// plane size (sml_set_payload_nt_threshold).
template <bool NT>
__device__ __forceinline__ void store_payload_as(u4* dst, u4 q) {
    if constexpr (NT) SML_NT_STORE16(q, dst);
    else *dst = q;
}

// ---------------------------------------------------- per-packet reductions

// Max of `m` over the P/4 lanes of this lane's packet (P <= 256).
// Inside each 16-lane row: four DPP steps (quad_perm xor 1, quad_perm xor 2,
// row_half_mirror, row_mirror) leave the row max in every lane of the row,
// with no LDS traffic.  Across rows: v_readlane of lanes 0/16/32/48 into
// SGPRs — for P >= 256 the packet max is then wave-uniform (scalar).
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

template <int P>
__device__ __forceinline__ uint32_t group_max(uint32_t m) {
    static_assert(P == 64 || P == 128 || P == 256, "row-based reduce covers 16..64 lanes");
    m = umax(m, dpp<0xB1>(m));    // quad_perm [1,0,3,2]
    m = umax(m, dpp<0x4E>(m));    // quad_perm [2,3,0,1]
    m = umax(m, dpp<0x141>(m));   // row_half_mirror
    m = umax(m, dpp<0x140>(m));   // row_mirror
    if constexpr (P == 64) return m;
    const uint32_t r0 = __builtin_amdgcn_readlane(m, 0), r1 = __builtin_amdgcn_readlane(m, 16);
    const uint32_t r2 = __builtin_amdgcn_readlane(m, 32), r3 = __builtin_amdgcn_readlane(m, 48);
    if constexpr (P == 128) return (threadIdx.x & 32) ? umax(r2, r3) : umax(r0, r1);
    return umax(umax(r0, r1), umax(r2, r3));
}

__device__ __forceinline__ uint32_t max4(f4 v) {
    uint32_t a = absbits(v.x), b = absbits(v.y), c = absbits(v.z), d = absbits(v.w);
    a = a > b ? a : b;
    c = c > d ? c : d;
    return a > c ? a : c;
}

// Exponents e[u] of the packet each lane's slice u belongs to (a tile of U
// slices; a packet of P > 256 elements is P / 256 consecutive slices).
template <int P, int U>
__device__ __forceinline__ void tile_exponents(const f4 (&v)[U], int (&e)[U]) {
    static_assert(P == 64 || P == 128 || P == 256 || P == 512 || P == 1024,
                  "packet_numel must be 64..1024, power of two");
    static_assert(P <= 256 * U, "a packet must lie inside one tile");
    uint32_t m[U];
#pragma unroll
    for (int u = 0; u < U; u++) m[u] = max4(v[u]);
    if constexpr (P <= 256) {
#pragma unroll
        for (int u = 0; u < U; u++) e[u] = exponent_of(group_max<P>(m[u]));
    } else {
        constexpr int G = P / 256;             // slices per packet
#pragma unroll
        for (int g = 0; g < U; g += G) {
            uint32_t t = m[g];
#pragma unroll
            for (int i = 1; i < G; i++) t = t > m[g + i] ? t : m[g + i];
            const int x = exponent_of(group_max<256>(t));
#pragma unroll
            for (int i = 0; i < G; i++) e[g + i] = x;
        }
    }
}

// The lane that owns packet `pkt` of slice u writes its exponent byte.
template <int P, int U>
__device__ __forceinline__ void store_exponents(int8_t* exps_out, uint64_t tile_base, int lane,
                                                const int (&e)[U], uint64_t nblocks) {
#pragma unroll
    for (int u = 0; u < U; u++) {
        bool leader;
        if constexpr (P <= 256) leader = (lane % (P / 4)) == 0;
        else leader = lane == 0 && (u % (P / 256)) == 0;
        uint64_t pkt = (tile_base + (uint64_t)(u * kWave + lane) * 4) / P;
        if (leader && pkt < nblocks) exps_out[pkt] = (int8_t)e[u];
    }
}

// A full tile's kPk = 256 U / P exponent bytes are contiguous in exps_out:
// lane 0 gathers them (v_readlane of each packet's first lane) and writes them
// with one 1/2/4/8/16-byte store — per-packet byte stores cost ~10 % on the
// 256 MiB bucket (partial-line writes).  dst must be kPk-byte aligned.
template <int P, int U>
__device__ __forceinline__ void store_tile_exponents(int8_t* dst, int lane, const int (&e)[U]) {
    constexpr int kPk = tile_elems<U>() / P;
    constexpr int kLanesPerPk = P / 4 < kWave ? P / 4 : kWave;
    constexpr int kWords = (kPk + 3) / 4;
    uint32_t w[kWords];
#pragma unroll
    for (int i = 0; i < kWords; i++) w[i] = 0;
#pragma unroll
    for (int j = 0; j < kPk; j++) {
        const int u = (j * P) / 256;
        uint32_t ej = 0;
#pragma unroll
        for (int uu = 0; uu < U; uu++)
            if (uu == u) ej = (uint32_t)__builtin_amdgcn_readlane(e[uu], (j * kLanesPerPk) % kWave);
        w[j / 4] |= (ej & 0xffu) << (8 * (j % 4));
    }
    if (lane != 0) return;
    if constexpr (kPk == 16) *reinterpret_cast<u4*>(dst) = mku4(w[0], w[1], w[2], w[3]);
    else if constexpr (kPk == 8) *reinterpret_cast<u2*>(dst) = u2{w[0], w[1]};
    else if constexpr (kPk == 4) *reinterpret_cast<uint32_t*>(dst) = w[0];
    else if constexpr (kPk == 2) *reinterpret_cast<uint16_t*>(dst) = (uint16_t)w[0];
    else *dst = (int8_t)w[0];
}

// Exponent byte of each lane's packet in slice u of a tile, with one
// wave-uniform scalar load per slice (base must be wave-uniform).  A slice
// holds 4, 2 or 1 packets (P = 64, 128, >= 256); their bytes lie in one
// aligned dword whenever exps is 4-byte aligned, and always for P > 256.
template <int P>
__device__ __forceinline__ bool slice_exps_scalar_ok(const int8_t* exps) {
    return P > 256 || (reinterpret_cast<uintptr_t>(exps) & 3u) == 0;
}
template <int P>
__device__ __forceinline__ uint32_t slice_exponent_byte(const int8_t* exps, uint64_t base, int u, int lane) {
    const uintptr_t e0 = reinterpret_cast<uintptr_t>(exps);
    const uintptr_t first = e0 + base / P + (uint64_t)(u * 256) / P;
    const uint32_t word = *reinterpret_cast<ConstU32*>(first & ~(uintptr_t)3);
    const uintptr_t mine = e0 + (base + (uint64_t)(u * kWave + lane) * 4) / P;
    return (word >> (8 * (mine & 3u))) & 0xffu;
}

// scale_of for W = 2^k without the double division: 2147483647 / 2^(e+k)
// rounds to 2^(31-e-k) (normal range for every int8 e and k <= 16), +inf when
// 31-e-k > 127, and 0 when W * 2^e overflows float (e + k >= 128).
__device__ __forceinline__ float scale_of_pow2(uint32_t log2W, int e) {
    const int m = e + (int)log2W;
    if (m >= 128) return 0.0f;
    const int x = 31 - m;                      // result 2^x
    if (x > 127) return __builtin_huge_valf();
    return __uint_as_float((uint32_t)(x + 127) << 23);
}

// The scale every kernel uses (power-of-two W takes the division-free form).
__device__ __forceinline__ float scale_for(uint32_t W, int e) {
    return (W & (W - 1)) == 0 ? scale_of_pow2(31 - __builtin_clz(W), e) : scale_of(W, e);
}

// For W = 2^k the scale is a power of two (or +inf / 0), so its reciprocal is
// exact and q / s == q * (1 / s) bit for bit: both round the same real number
// q * 2^-x once (2^-x is representable for every x here, 2^-127 as a
// denormal); s = +inf -> 1/s = 0 and s = 0 -> 1/s = +inf give the same
// signed zeros / infinities / NaN as the division.
__device__ __forceinline__ float rcp_scale_pow2(uint32_t log2W, int e) {
    const int m = e + (int)log2W;
    if (m >= 128) return __builtin_huge_valf();  // scale 0
    const int x = 31 - m;
    if (x > 127) return 0.0f;                     // scale +inf
    return __builtin_ldexpf(1.0f, -x);
}

// Per-workgroup scale table, lut[(uint8_t)e], built once per launch-block.
// Reciprocal table for power-of-two W (dequantize by multiplication).
__device__ __forceinline__ void build_rcp_lut(float* lut, uint32_t W) {
    lut[threadIdx.x] = rcp_scale_pow2(31 - __builtin_clz(W), (int)(int8_t)(uint8_t)threadIdx.x);
    __syncthreads();
}

__device__ __forceinline__ void build_lut(float* lut, uint32_t W) {
    lut[threadIdx.x] = scale_for(W, (int)(int8_t)(uint8_t)threadIdx.x);
    __syncthreads();
}

// ------------------------------------------------------- launch geometry

// The wave's index in its workgroup, as a wave-uniform (SGPR) value, so that
// tile bases and per-tile metadata addresses are scalar.
__device__ __forceinline__ uint32_t wave_index() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// Workgroup -> data order for the HBM streams.  The dispatcher places
// workgroup b on XCD b % 8; with chunk C > 0 the first (nb / 8C) * 8C
// workgroups are permuted so that each XCD sweeps runs of C consecutive
// workgroups' data (C x 16 KiB with 4 tiles per workgroup) instead of every
// 8th one; the tail keeps its order (a bijection on [0, nb) either way).
// Measured on the 256 MiB bucket: C = 64 moves a 1:1 read:write stream
// 4 % faster than the plain order (profiles/r01/ab5_xcd_chunk.json, hbm_probe_*.json).
__device__ __forceinline__ uint64_t xcd_block(uint32_t C) {
    const uint64_t b = blockIdx.x;
    if (C == 0) return b;
    const uint64_t span = 8ull * C, full = (uint64_t)gridDim.x / span * span;
    if (b >= full) return b;
    const uint64_t r = b / 8;
    return (r / C) * span + (b % 8) * C + r % C;
}


struct QuantArgs {
    const float* in;
    uint64_t numel;
    uint64_t nblocks;       // B
    uint64_t ntiles;        // ceil(B*P / tile_elems<U>())
    const int8_t* gexp;     // global exponents (K3) or nullptr (K1)
    u4* payload;          // B*P words, 16-B aligned (nullptr: exponents only)
    int8_t* exps_out;       // nullable
    uint32_t W;
    uint32_t xcd;           // xcd_block chunk (0 = plain order)
};

template <bool ALIGNED, int U>
__device__ __forceinline__ void load_tile(const QuantArgs& a, uint64_t base, int lane, f4 (&v)[U]) {
    if (base + tile_elems<U>() <= a.numel) {
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

// Word stream in the quantizer's tile shape (1024 words per wave, 16-B
// non-temporal loads, default-policy stores, XCD order, one-shot grid; any
// 4-byte alignment; in may alias out): out[i] = op(in[i]).  K5 (loopback),
// the INT32 byteswap and the in-node switch's gather copy instantiate it.
template <class Op>
__global__ __launch_bounds__(kBlockThreads) void k_words(const uint32_t* in, uint32_t* out, uint64_t n, uint32_t xcd,
                                                         Op op) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t ntiles = (n + kTileElems - 1) / kTileElems;
    for (uint64_t t = xcd_block(xcd) * kWavesPerBlock + wave_index(); t < ntiles; t += nwaves) {
        const uint64_t base = t * kTileElems;
        if (base + kTileElems <= n) {
            u4a v[kU];
#pragma unroll
            for (int u = 0; u < kU; u++)
                v[u] = __builtin_nontemporal_load(reinterpret_cast<const u4a*>(in + base + (u * kWave + lane) * 4));
#pragma unroll
            for (int u = 0; u < kU; u++)
                *reinterpret_cast<u4a*>(out + base + (u * kWave + lane) * 4) =
                    u4a{op(v[u].x), op(v[u].y), op(v[u].z), op(v[u].w)};
        } else {
#pragma unroll
            for (int u = 0; u < kU; u++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4 + j;
                    if (idx < n) out[idx] = op(in[idx]);
                }
        }
    }
}

}  // namespace sml

#endif  // SML_DEVICE_H_
