// hbm_probe.hip — standalone HBM ceiling probe for the K1 access shape on
// gfx950 (tools only; not part of the product library).
//
// Question it answers: is K1's 6.8 TB/s (read 4N fp32 + write 4N int32) the
// ceiling for a 1:1 read:write stream on MI355X, or does another shape
// (workgroup size, f4 per lane, cache policy, XCD-contiguous block order,
// read-only / write-only) move more bytes?  Every variant is timed in every
// round (interleaved), medians reported as JSON on stdout.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o bin/hbm_probe tools/hbm_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

// LOADNT / STORENT: 0 default policy, 1 nontemporal.
// XCD: remap blockIdx so that each XCD (blockIdx % 8 under round-robin
// dispatch) sweeps contiguous runs of XCD blocks (-1: one contiguous eighth
// of the buffer per XCD; 0: no remap).
template <int WG, int U, int LOADNT, int STORENT, int XCD>
__global__ __launch_bounds__(WG) void k_copy(const u4* __restrict__ in, u4* __restrict__ out, unsigned long long nvec) {
    unsigned long long b = blockIdx.x;
    if (XCD < 0) {
        const unsigned long long nb = gridDim.x, per = nb / 8;
        b = (b % 8) * per + b / 8;   // nb is a multiple of 8
    } else if (XCD > 0) {
        const unsigned long long r = b / 8;   // this XCD's r-th block
        b = (r / XCD) * 8 * XCD + (b % 8) * XCD + r % XCD;
    }
    const unsigned long long base = b * (unsigned long long)(WG * U) + (threadIdx.x / 64) * (64ull * U) + (threadIdx.x % 64);
    u4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const u4* p = in + base + 64ull * u;
        v[u] = LOADNT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        v[u].x ^= 0x80000000u;       // touch the data (like a quantizer would)
        u4* p = out + base + 64ull * u;
        if (STORENT) __builtin_nontemporal_store(v[u], p); else *p = v[u];
    }
    (void)nvec;
}

// Copy with the destination shifted by OFF bytes (unaligned 16-B stores, as
// at the 52-byte payload offset of a DPDK frame).
typedef unsigned int u4a __attribute__((ext_vector_type(4), aligned(4)));
template <int OFF>
__global__ __launch_bounds__(256) void k_copy_off(const u4* __restrict__ in, unsigned char* __restrict__ out) {
    const unsigned long long r = blockIdx.x / 8, C = 64, span = 8 * C;
    unsigned long long b = blockIdx.x;
    if (b < gridDim.x / span * span) b = (r / C) * span + (b % 8) * C + r % C;
    const unsigned long long base = b * 1024ull + (threadIdx.x / 64) * 256ull + (threadIdx.x % 64);
    u4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = __builtin_nontemporal_load(in + base + 64ull * u);
#pragma unroll
    for (int u = 0; u < 4; u++) {
        u4a w = {v[u].x ^ 1u, v[u].y, v[u].z, v[u].w};
        *reinterpret_cast<u4a*>(out + OFF + 16ull * (base + 64ull * u)) = w;
    }
}

// Copy with the SOURCE shifted by OFF bytes (unaligned 16-B loads, as when
// reading payloads at the 52-byte offset of returned frames).
template <int OFF, int NT>
__global__ __launch_bounds__(256) void k_copy_srcoff(const unsigned char* __restrict__ in, u4* __restrict__ out) {
    const unsigned long long r = blockIdx.x / 8, C = 64, span = 8 * C;
    unsigned long long b = blockIdx.x;
    if (b < gridDim.x / span * span) b = (r / C) * span + (b % 8) * C + r % C;
    const unsigned long long base = b * 1024ull + (threadIdx.x / 64) * 256ull + (threadIdx.x % 64);
    u4a v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const u4a* p = reinterpret_cast<const u4a*>(in + OFF + 16ull * (base + 64ull * u));
        v[u] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        u4 w = {v[u].x ^ 1u, v[u].y, v[u].z, v[u].w};
        out[base + 64ull * u] = w;
    }
}

// Fewer, longer-lived workgroups: each processes ITER consecutive 16 KiB
// chunks (wg256 x 4 f4 per lane per chunk), loads of chunk i+1 issued before
// the stores of chunk i; XCD order over workgroups (runs of C).
template <int ITER, int C>
__global__ __launch_bounds__(256) void k_copy_multi(const u4* __restrict__ in, u4* __restrict__ out) {
    const unsigned long long r = blockIdx.x / 8, span = 8ull * C;
    unsigned long long b = blockIdx.x;
    if (b < gridDim.x / span * span) b = (r / C) * span + (b % 8) * C + r % C;
    const unsigned long long base0 = b * (1024ull * ITER) + (threadIdx.x / 64) * 256ull + (threadIdx.x % 64);
    u4 v[4], w[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = __builtin_nontemporal_load(in + base0 + 64ull * u);
#pragma unroll
    for (int it = 0; it < ITER; it++) {
        const unsigned long long base = base0 + 1024ull * it;
        if (it + 1 < ITER) {
#pragma unroll
            for (int u = 0; u < 4; u++) w[u] = __builtin_nontemporal_load(in + base + 1024 + 64ull * u);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            u4 x = v[u];
            x.x ^= 0x80000000u;
            out[base + 64ull * u] = x;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = w[u];
    }
}

template <int WG, int U, int LOADNT>
__global__ __launch_bounds__(WG) void k_read(const u4* __restrict__ in, unsigned int* __restrict__ sink) {
    const unsigned long long base = blockIdx.x * (unsigned long long)(WG * U) + (threadIdx.x / 64) * (64ull * U) + (threadIdx.x % 64);
    unsigned int acc = 0;
    u4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const u4* p = in + base + 64ull * u;
        v[u] = LOADNT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < U; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;   // practically never: keeps the loads
}

template <int WG, int U, int STORENT>
__global__ __launch_bounds__(WG) void k_write(u4* __restrict__ out) {
    const unsigned long long base = blockIdx.x * (unsigned long long)(WG * U) + (threadIdx.x / 64) * (64ull * U) + (threadIdx.x % 64);
#pragma unroll
    for (int u = 0; u < U; u++) {
        u4 v = {(unsigned)base, (unsigned)u, 1u, 2u};
        u4* p = out + base + 64ull * u;
        if (STORENT) __builtin_nontemporal_store(v, p); else *p = v;
    }
}

// Round 4: explicit cache-policy bits on buffer loads / stores (aux: 1 sc0,
// 2 nt, 16 sc1; __builtin_nontemporal_* emit nt alone).  One descriptor per
// workgroup over its own 16 KiB (WG 256 x U 4), so offsets stay 32-bit.
template <int LAUX, int SAUX>
__global__ __launch_bounds__(256) void k_copy_cp(const u4* __restrict__ in, u4* __restrict__ out) {
    const unsigned long long r = blockIdx.x / 8, C = 64, span = 8 * C;
    unsigned long long b = blockIdx.x;
    if (b < gridDim.x / span * span) b = (r / C) * span + (b % 8) * C + r % C;
    const unsigned long long wgb = b * 1024ull;   // u4 index of this workgroup's 16 KiB
    __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void*)(in + wgb), 0, 16384, 0x00020000);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)(out + wgb), 0, 16384, 0x00020000);
    const int off = ((threadIdx.x / 64) * 256 + (threadIdx.x % 64)) * 16;
    u4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = __builtin_amdgcn_raw_buffer_load_b128(ri, off + 1024 * u, 0, LAUX);
#pragma unroll
    for (int u = 0; u < 4; u++) {
        v[u].x ^= 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(v[u], ro, off + 1024 * u, 0, SAUX);
    }
}

template <int SAUX>
__global__ __launch_bounds__(256) void k_write_cp(u4* __restrict__ out) {
    const unsigned long long wgb = blockIdx.x * 1024ull;
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)(out + wgb), 0, 16384, 0x00020000);
    const int off = ((threadIdx.x / 64) * 256 + (threadIdx.x % 64)) * 16;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        u4 v = {(unsigned)wgb, (unsigned)u, 1u, 2u};
        __builtin_amdgcn_raw_buffer_store_b128(v, ro, off + 1024 * u, 0, SAUX);
    }
}

struct Variant {
    std::string name;
    double bytes_per_vec;   // bytes moved per 16-B vector of the buffer
    std::function<void(hipStream_t)> launch;
    std::vector<float> us;
};

int main(int argc, char** argv) {
    const unsigned long long bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 256ull) << 20;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const int reps = 10;
    const unsigned long long nvec = bytes / 16;
    u4 *in, *out;
    unsigned int* sink;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&out, bytes));
    u4* out2;
    CK(hipMalloc(&out2, bytes + 4096));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(in, 1, bytes));
    CK(hipMemset(out, 0, bytes));
    hipStream_t st;
    CK(hipStreamCreate(&st));

    std::vector<Variant> vs;
#define COPY(WG, U, LN, SN, X) vs.push_back({"copy wg" #WG " u" #U " ldnt" #LN " stnt" #SN " xcd" #X, 32.0, \
    [=](hipStream_t s) { unsigned long long g = nvec / (WG * U); \
        k_copy<WG, U, LN, SN, X><<<g, WG, 0, s>>>(in, out, nvec); }, {}})
#define READ(WG, U, LN) vs.push_back({"read wg" #WG " u" #U " ldnt" #LN, 16.0, \
    [=](hipStream_t s) { unsigned long long g = nvec / (WG * U); k_read<WG, U, LN><<<g, WG, 0, s>>>(in, sink); }, {}})
#define WRITE(WG, U, SN) vs.push_back({"write wg" #WG " u" #U " stnt" #SN, 16.0, \
    [=](hipStream_t s) { unsigned long long g = nvec / (WG * U); k_write<WG, U, SN><<<g, WG, 0, s>>>(out); }, {}})
#define MULTI(IT, C) vs.push_back({"copy multi iter" #IT " xcd" #C, 32.0, \
    [=](hipStream_t s) { k_copy_multi<IT, C><<<nvec / (1024 * IT), 256, 0, s>>>(in, out); }, {}})
#define COPYCP(L, S) vs.push_back({"copy cpol load" #L " store" #S, 32.0, \
    [=](hipStream_t s) { k_copy_cp<L, S><<<nvec / 1024, 256, 0, s>>>(in, out); }, {}})
#define WRITECP(S) vs.push_back({"write cpol store" #S, 16.0, \
    [=](hipStream_t s) { k_write_cp<S><<<nvec / 1024, 256, 0, s>>>(out); }, {}})
    const char* set = getenv("PROBE_SET");
    if (set && std::string(set) == "tiles") {
        // tile size (U f4 per lane) x workgroup size x XCD run length
        COPY(256, 4, 1, 0, 64);  // == K1 now
        COPY(256, 4, 1, 0, 32);
        COPY(128, 4, 1, 0, 128);
        COPY(256, 2, 1, 0, 64);
        COPY(256, 2, 1, 0, 128);
        COPY(128, 2, 1, 0, 128);
        COPY(128, 2, 1, 0, 256);
        COPY(64, 2, 1, 0, 256);
        COPY(64, 2, 1, 0, 512);
        COPY(64, 4, 1, 0, 256);
        COPY(256, 1, 1, 0, 256);
        READ(256, 4, 1);
        WRITE(256, 4, 0);
    } else if (set && std::string(set) == "nt") {
        // round 4: the read-only and write-only rates behind the copy
        // ceiling, with K1's store policy (non-temporal) and tile shapes
        COPY(256, 4, 1, 1, 64);
        COPY(256, 2, 1, 1, 64);
        COPY(256, 4, 1, 0, 64);
        READ(256, 4, 1);
        READ(256, 2, 1);
        WRITE(256, 4, 1);
        WRITE(256, 2, 1);
        WRITE(256, 4, 0);
    } else if (set && std::string(set) == "cpol") {
        // round 4: store (and load) cache-policy bits beyond nt; aux 1 sc0,
        // 2 nt, 16 sc1
        COPY(256, 4, 1, 1, 64);   // K1's policy through global_* (reference row)
        COPYCP(2, 2);
        COPYCP(2, 0);
        COPYCP(2, 1);
        COPYCP(2, 3);
        COPYCP(2, 16);
        COPYCP(2, 17);
        COPYCP(2, 18);
        COPYCP(2, 19);
        COPYCP(0, 2);
        COPYCP(19, 2);
        COPYCP(3, 2);
        WRITE(256, 4, 1);
        WRITECP(2);
        WRITECP(0);
        WRITECP(1);
        WRITECP(3);
        WRITECP(16);
        WRITECP(17);
        WRITECP(18);
        WRITECP(19);
    } else {
        COPY(256, 4, 1, 0, 64);  // == K1 now
        MULTI(1, 64);
        MULTI(2, 32);
        MULTI(4, 16);
        MULTI(8, 8);
        MULTI(16, 4);
        MULTI(2, 64);
        MULTI(4, 64);
        READ(256, 4, 1);
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto& v : vs) { v.launch(st); }
    CK(hipStreamSynchronize(st));
    for (int r = 0; r < rounds; r++) {
        for (auto& v : vs) {
            v.launch(st);
            CK(hipEventRecord(a, st));
            for (int i = 0; i < reps; i++) v.launch(st);
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            v.us.push_back(ms * 1000.f / reps);
        }
        fprintf(stderr, "round %d done\n", r);
    }
    CK(hipGetLastError());
    printf("{\"bytes\": %llu, \"rounds\": %d, \"reps\": %d, \"variants\": [", bytes, rounds, reps);
    for (size_t i = 0; i < vs.size(); i++) {
        auto& v = vs[i];
        std::sort(v.us.begin(), v.us.end());
        const double med = v.us[v.us.size() / 2];
        const double moved = v.bytes_per_vec * nvec;   // copy: 2x buffer, read/write: 1x
        printf("%s{\"name\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"GBps\": %.1f}", i ? ", " : "",
               v.name.c_str(), med, v.us[0], moved / med * 1e-3);
    }
    printf("]}\n");
    return 0;
}
