/*
 * sml_oracle.c — CPU restatement of SwitchML's end-host pre/post-processor
 * (CpuExponentQuantizerPPP, VCL=0 build) and of the dummy-backend packet loop
 * that drives it.
 *
 * TEST INFRASTRUCTURE ONLY — see sml_oracle.h for who may call this and for
 * its parity status ("parity unpinned" at the bit level: the reference is not
 * buildable in this image; pinned by the reference's 1 % known-answer checks
 * and hand-derived vectors).
 *
 * Citations are relative to /root/reference/dev_root/client_lib/src/.
 */
#include "sml_oracle.h"

#include <emmintrin.h> /* SSE2: the instruction set the reference's VCL=1 build targets */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static inline uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

uint64_t orc_num_blocks(uint64_t numel, uint64_t P) {
    /* ppp.cc:56-57: tensor_size = numel * DataTypeSize; (size + ltu - 1) / ltu */
    uint64_t bytes = numel * 4, ltu = P * 4;
    return (bytes + ltu - 1) / ltu;
}

int8_t orc_block_exponent(const float* x, uint64_t n) {
    /* ppp.cc:129-146 (scalar loop): current_max starts at 0; v = abs(x);
     * if (v > current_max) current_max = v.  NaN compares false: never taken. */
    float current_max = 0.0f;
    for (uint64_t i = 0; i < n; i++) {
        float v = fabsf(x[i]);
        if (v > current_max) current_max = v;
    }
    /* ppp.cc:154: ((bits & 0x7f800000) >> 23) - 126, stored through int8_t* */
    int32_t bits = (int32_t)f2u(current_max);
    int32_t e = ((bits & 0x7f800000) >> 23) - 126;
    return (int8_t)(uint8_t)(e & 0xff);
}

float orc_scale(uint16_t num_workers, int8_t exponent) {
    /* ppp.cc:257-258: scaling_factors_[ltu] =
     *   double(INT32_MAX) / (num_workers * powf(2, exponent));
     * num_workers (uint16) * float -> float multiply; the quotient is a double
     * and is rounded to float on store. */
    float denom = (float)num_workers * powf(2.0f, (float)exponent);
    double q = (double)2147483647 / (double)denom;
    return (float)q;
}

void orc_scale_lut(uint16_t num_workers, float lut[256]) {
    for (int i = 0; i < 256; i++) lut[i] = orc_scale(num_workers, (int8_t)(uint8_t)i);
}

/* gcc x86-64 lowers the (UB for negatives) float -> uint32_t conversion of
 * ppp.cc:103 as cvttss2si %xmm, %rax (64-bit signed truncation) and keeps the
 * low 32 bits.  Out-of-int64-range or NaN gives the "integer indefinite"
 * 0x8000000000000000, whose low half is 0. */
static inline uint32_t x86_f2u32(float r) {
    if (!(fabsf(r) < 0x1p63f)) return 0u;
    return (uint32_t)(uint64_t)(int64_t)r;
}

uint32_t orc_quantize_value(float x, float scale) {
    /* ppp.cc:103: out_ptr[i] = htonl(std::round(in_ptr[i] * scaling_factors_[ltu_id])); */
    float prod = x * scale;           /* float * float, correctly rounded */
    float r = roundf(prod);           /* std::round(float): half away from zero */
    return bswap32(x86_f2u32(r));     /* htonl on little-endian */
}

uint32_t orc_quantize_value_rne(float x, float scale) {
    /* VCL=1 body (ppp.cc:96-98): roundi() = cvtps2dq under the default MXCSR
     * (round-to-nearest-even); out of int32 range or NaN -> 0x80000000. */
    float prod = x * scale;
    uint32_t q;
    if (!(fabsf(prod) < 0x1p31f)) {
        q = 0x80000000u;
    } else {
        float r = nearbyintf(prod); /* default rounding mode is RNE */
        q = (uint32_t)(int32_t)r;
    }
    return bswap32(q);
}

float orc_dequantize_value(uint32_t be_word, float scale) {
    /* ppp.cc:240-241: int32_t in_be = (int32_t) ntohl(in_ptr[j]);
     *                 out_ptr[j] = in_be / scaling_factors_[ltu_id];
     * int -> float conversion (RNE) then IEEE float division. */
    int32_t v = (int32_t)bswap32(be_word);
    return (float)v / scale;
}

void orc_exponents(const float* in, uint64_t numel, uint64_t P, int8_t* exps) {
    uint64_t B = orc_num_blocks(numel, P);
    for (uint64_t k = 0; k < B; k++) {
        uint64_t off = k * P, n = numel - off < P ? numel - off : P;
        exps[k] = orc_block_exponent(in + off, n);
    }
}

void orc_quantize(const float* in, uint64_t numel, uint64_t P, uint16_t num_workers,
                  const int8_t* global_exps, int rounding, uint32_t* payload_be) {
    uint64_t B = orc_num_blocks(numel, P);
    float lut[256];
    orc_scale_lut(num_workers, lut);
    for (uint64_t k = 0; k < B; k++) {
        uint64_t off = k * P, n = numel - off < P ? numel - off : P;
        int8_t e = global_exps ? global_exps[k] : orc_block_exponent(in + off, n);
        float s = lut[(uint8_t)e];
        uint64_t i = 0;
        if (rounding == 1) {
            /* VCL body covers n - n % 16 elements (ppp.cc:92-99), scalar tail after. */
            uint64_t vec = n - n % 16;
            for (; i < vec; i++) payload_be[off + i] = orc_quantize_value_rne(in[off + i], s);
        }
        for (; i < n; i++) payload_be[off + i] = orc_quantize_value(in[off + i], s);
        for (; i < P; i++) payload_be[off + i] = 0u; /* reference: stale ring bytes */
    }
}

void orc_dequantize(const uint32_t* payload_be, const int8_t* global_exps, uint64_t numel,
                    uint64_t P, uint16_t num_workers, float* out) {
    uint64_t B = orc_num_blocks(numel, P);
    float lut[256];
    orc_scale_lut(num_workers, lut);
    for (uint64_t k = 0; k < B; k++) {
        uint64_t off = k * P, n = numel - off < P ? numel - off : P;
        float s = lut[(uint8_t)global_exps[k]];
        for (uint64_t i = 0; i < n; i++) out[off + i] = orc_dequantize_value(payload_be[off + i], s);
    }
}

void orc_bswap32(const uint32_t* in, uint32_t* out, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) out[i] = bswap32(in[i]);
}

void orc_loopback_aggregate(uint32_t* payload_be, uint64_t n, uint16_t num_workers) {
    /* dummy_backend.cc:78-82: SWAP_INT32, *= num_workers (int32 wrap), SWAP_INT32 */
    for (uint64_t j = 0; j < n; j++) {
        uint32_t v = bswap32(payload_be[j]);
        v = v * (uint32_t)num_workers;
        payload_be[j] = bswap32(v);
    }
}

void orc_switch_exps(const int8_t* const* exps, int W, uint64_t B, int8_t* out) {
    /* exponents.p4:48-54: signed max over workers of int<8> */
    for (uint64_t k = 0; k < B; k++) {
        int8_t m = exps[0][k];
        for (int w = 1; w < W; w++) if (exps[w][k] > m) m = exps[w][k];
        out[k] = m;
    }
}

void orc_switch_payload(const uint32_t* const* payload_be, int W, uint64_t n, uint32_t* out) {
    /* processor.p4:48-54: value = value + worker value as bit<32> (wrapping);
     * the switch parses the payload big-endian and emits big-endian. */
    for (uint64_t j = 0; j < n; j++) {
        uint32_t acc = 0;
        for (int w = 0; w < W; w++) acc += bswap32(payload_be[w][j]);
        out[j] = bswap32(acc);
    }
}

void orc_slice(uint64_t numel, int T, int t, uint64_t* offset, uint64_t* slice_numel) {
    /* fifo_scheduler.cc:93-109 */
    uint64_t n = numel / (uint64_t)T;
    uint64_t rem = numel % (uint64_t)T;
    if (rem > (uint64_t)t) {
        n++;
        *offset = (uint64_t)t * n;
    } else {
        *offset = (uint64_t)t * n + rem;
    }
    *slice_numel = n;
}

/* ------------------------------------------------------------------------ */
/* Packet-loop restatement: one PPP instance per worker thread.              */

typedef struct {
    const float* in;
    float* out;
    uint64_t numel;   /* slice numel */
    uint64_t P;       /* ltu numel */
    uint64_t B;       /* total_main_num_ltus_ (ppp.cc:57) */
    uint64_t b;       /* batch_num_ltus_ (ppp.cc:58) */
    uint16_t W;
    float* scales;    /* scaling_factors_ (ppp.cc:60) */
    const float* lut;
    int vcl;          /* 1: the VCL=1 build's vector loops (ppp.cc:88-99, 128-140) */
} orc_ppp;

/* ---- VCL=1 build, restated for the instruction set it is compiled for ----
 * client_lib/Makefile:113-120 adds -DVCL and no -m flags, so VCL's
 * instrset selection (un-vendored: github.com/vectorclass/version2) builds
 * for the x86-64 baseline, SSE2: Vec16f is four __m128.  Per 16 elements:
 *   quantize (ppp.cc:92-99): roundi(x * s) = cvtps2dq (RNE; out of range or
 *     NaN -> 0x80000000), then permute64<ENDIANESS_CONVERSION> = bswap32 of
 *     every word (SSE2 has no pshufb: shifts, masks, or);
 *   exponent scan (ppp.cc:128-140): max(acc, abs(x)) = maxps, then
 *     horizontal_max.
 * The tails (n % 16 elements) run the scalar loops, as in the reference.
 * Only the timing baseline and the RNE-mode cross-check use this; its bits
 * equal orc_quantize(rounding = 1) (tested), and like that mode it is parity
 * unpinned (VCL is not in /root/reference). */
static inline __m128i bswap32_sse2(__m128i v) {
    __m128i t = _mm_or_si128(_mm_slli_epi16(v, 8), _mm_srli_epi16(v, 8));   /* swap bytes in 16-bit halves */
    return _mm_or_si128(_mm_slli_epi32(t, 16), _mm_srli_epi32(t, 16));       /* swap the halves */
}

static void vcl_quantize_block(const float* in, uint64_t n, float sc, uint32_t* out) {
    const __m128 s = _mm_set1_ps(sc);
    uint64_t i = 0, vec = n - n % 16;
    for (; i < vec; i += 4) {
        __m128i q = _mm_cvtps_epi32(_mm_mul_ps(_mm_loadu_ps(in + i), s));
        _mm_storeu_si128((__m128i*)(out + i), bswap32_sse2(q));
    }
    for (; i < n; i++) out[i] = orc_quantize_value(in[i], sc);
}

static int8_t vcl_block_exponent(const float* x, uint64_t n) {
    const __m128 absmask = _mm_castsi128_ps(_mm_set1_epi32(0x7fffffff));
    __m128 acc = _mm_setzero_ps();
    uint64_t i = 0, vec = n - n % 16;
    for (; i < vec; i += 4) acc = _mm_max_ps(acc, _mm_and_ps(_mm_loadu_ps(x + i), absmask));
    float current_max = 0.0f;
    if (vec) { /* horizontal_max */
        acc = _mm_max_ps(acc, _mm_movehl_ps(acc, acc));
        acc = _mm_max_ss(acc, _mm_shuffle_ps(acc, acc, 1));
        current_max = _mm_cvtss_f32(acc);
    }
    for (; i < n; i++) {
        float v = fabsf(x[i]);
        if (v > current_max) current_max = v;
    }
    int32_t bits = (int32_t)f2u(current_max);
    int32_t e = ((bits & 0x7f800000) >> 23) - 126;
    return (int8_t)(uint8_t)(e & 0xff);
}

void orc_quantize_vcl(const float* in, uint64_t numel, uint64_t P, uint16_t num_workers, uint32_t* payload_be,
                      int8_t* exps) {
    uint64_t B = orc_num_blocks(numel, P);
    float lut[256];
    orc_scale_lut(num_workers, lut);
    for (uint64_t k = 0; k < B; k++) {
        uint64_t off = k * P, n = numel - off < P ? numel - off : P;
        int8_t e = vcl_block_exponent(in + off, n);
        exps[k] = e;
        vcl_quantize_block(in + off, n, lut[(uint8_t)e], payload_be + off);
        for (uint64_t i = n; i < P; i++) payload_be[off + i] = 0u;
    }
}

/* PreprocessSingle, FLOAT32 branch — ppp.cc:69-156 */
static void ppp_preprocess(orc_ppp* s, uint64_t ltu_id, uint32_t* entries, uint8_t* extra) {
    if (ltu_id >= s->b) {
        uint64_t k = ltu_id - s->b;
        uint64_t off = k * s->P;
        uint64_t n = s->numel - off < s->P ? s->numel - off : s->P;
        float sc = s->scales[k];
        if (s->vcl) vcl_quantize_block(s->in + off, n, sc, entries);
        else for (uint64_t i = 0; i < n; i++) entries[i] = orc_quantize_value(s->in[off + i], sc);
        ltu_id = k + s->b;
    }
    if (ltu_id < s->B) {
        uint64_t off = ltu_id * s->P;
        uint64_t n = s->numel - off < s->P ? s->numel - off : s->P;
        extra[0] = (uint8_t)(s->vcl ? vcl_block_exponent(s->in + off, n) : orc_block_exponent(s->in + off, n));
    }
}

/* PostprocessSingle, FLOAT32 branch — ppp.cc:194-260 */
static void ppp_postprocess(orc_ppp* s, uint64_t ltu_id, const uint32_t* entries, const uint8_t* extra) {
    if (ltu_id >= s->b) {
        uint64_t k = ltu_id - s->b;
        uint64_t off = k * s->P;
        uint64_t n = s->numel - off < s->P ? s->numel - off : s->P;
        float sc = s->scales[k];
        for (uint64_t i = 0; i < n; i++) s->out[off + i] = orc_dequantize_value(entries[i], sc);
        ltu_id = k + s->b;
    }
    if (ltu_id < s->B) s->scales[ltu_id] = s->lut[extra[0]];
}

typedef struct {
    orc_ppp ppp;
    int mode;
    int8_t* pkt_exps;       /* optional stream capture */
    uint32_t* pkt_payload;  /* optional stream capture */
    int rc;
} orc_worker;

/* Record packet p as sent: the exponent byte if p < B, the payload words of
 * block p-b if p >= b; everything the reference leaves stale is recorded as 0. */
static void capture(orc_worker* w, uint64_t p, const uint32_t* ent, const uint8_t* ex) {
    const orc_ppp* s = &w->ppp;
    w->pkt_exps[p] = p < s->B ? (int8_t)ex[0] : 0;
    uint32_t* dst = w->pkt_payload + p * s->P;
    memset(dst, 0, s->P * 4);
    if (p >= s->b) {
        uint64_t off = (p - s->b) * s->P;
        uint64_t n = s->numel - off < s->P ? s->numel - off : s->P;
        memcpy(dst, ent, n * 4);
    }
}

/* DummyWorkerThread::operator() main loop for one slice, in-order delivery
 * (dummy_worker_thread.cc:86-177; ReceiveBurst's random order does not change
 * results: packet p only needs scale[p-b], stored when packet p-b returned). */
static void* worker_run(void* arg) {
    orc_worker* w = (orc_worker*)arg;
    orc_ppp* s = &w->ppp;
    w->rc = 0;
    if (s->numel == 0) return NULL; /* dummy_worker_thread.cc:87 */
    uint64_t total = s->B + s->b;   /* NeedsExtraBatch() for FLOAT32 (:95-99) */
    uint32_t* ring = (uint32_t*)calloc(s->b * s->P, 4);
    uint8_t* extra = (uint8_t*)calloc(s->b * 2, 1);
    s->scales = (float*)malloc(s->B * sizeof(float));
    if (!ring || !extra || !s->scales) { w->rc = -1; goto done; }

    for (uint64_t p = 0; p < s->b; p++) { /* first batch (:106-116) */
        ppp_preprocess(s, p, ring + (p % s->b) * s->P, extra + (p % s->b) * 2);
        if (w->pkt_exps) capture(w, p, ring + (p % s->b) * s->P, extra + (p % s->b) * 2);
    }
    for (uint64_t p = 0; p < total; p++) { /* receive loop (:126-177), in order */
        uint32_t* ent = ring + (p % s->b) * s->P;
        uint8_t* ex = extra + (p % s->b) * 2;
        if (w->mode == ORC_MODE_ROUNDTRIP) {
            orc_loopback_aggregate(ent, s->P, s->W); /* ProcessPacket (dummy_backend.cc:72-84) */
            ppp_postprocess(s, p, ent, ex);
        } else if (p < s->B) {
            s->scales[p] = s->lut[ex[0]]; /* the scale-store half of PostprocessSingle */
        }
        uint64_t np = p + s->b;
        if (np >= total) continue;
        ppp_preprocess(s, np, ent, ex);
        if (w->pkt_exps) capture(w, np, ent, ex);
    }
done:
    free(ring);
    free(extra);
    free(s->scales);
    s->scales = NULL;
    return NULL;
}

int orc_dummy_allreduce(const float* in, float* out, uint64_t numel, uint64_t P,
                        uint32_t max_outstanding_packets, int T, uint16_t W,
                        int threaded, int mode) {
    return orc_dummy_allreduce_ex(in, out, numel, P, max_outstanding_packets, T, W, threaded, mode, 0);
}

int orc_dummy_allreduce_ex(const float* in, float* out, uint64_t numel, uint64_t P,
                           uint32_t max_outstanding_packets, int T, uint16_t W,
                           int threaded, int mode, int vcl) {
    if (T <= 0 || P == 0) return -1;
    float lut[256];
    orc_scale_lut(W, lut);
    orc_worker* ws = (orc_worker*)calloc((size_t)T, sizeof(orc_worker));
    pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
    if (!ws || !th) { free(ws); free(th); return -1; }
    uint64_t batch_max = max_outstanding_packets / (uint64_t)T; /* dummy_worker_thread.cc:59 */
    for (int t = 0; t < T; t++) {
        uint64_t off, n;
        orc_slice(numel, T, t, &off, &n);
        orc_ppp* s = &ws[t].ppp;
        s->in = in + off;
        s->out = out + off;
        s->numel = n;
        s->P = P;
        s->B = orc_num_blocks(n, P);
        s->b = s->B < batch_max ? s->B : batch_max;
        s->W = W;
        s->lut = lut;
        s->vcl = vcl;
        ws[t].mode = mode;
        if (s->b == 0 && s->B > 0) { free(ws); free(th); return -1; }
    }
    int rc = 0;
    if (threaded && T > 1) {
        for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, worker_run, &ws[t]);
        for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    } else {
        for (int t = 0; t < T; t++) worker_run(&ws[t]);
    }
    for (int t = 0; t < T; t++) rc |= ws[t].rc;
    free(ws);
    free(th);
    return rc;
}

int orc_dummy_packet_stream(const float* in, uint64_t numel, uint64_t P, uint32_t batch_max,
                            uint16_t W, int8_t* pkt_exps, uint32_t* pkt_payload, float* out) {
    float lut[256];
    orc_scale_lut(W, lut);
    orc_worker w;
    memset(&w, 0, sizeof(w));
    w.ppp.in = in;
    w.ppp.out = out;
    w.ppp.numel = numel;
    w.ppp.P = P;
    w.ppp.B = orc_num_blocks(numel, P);
    w.ppp.b = w.ppp.B < batch_max ? w.ppp.B : batch_max;
    w.ppp.W = W;
    w.ppp.lut = lut;
    w.mode = ORC_MODE_ROUNDTRIP;
    w.pkt_exps = pkt_exps;
    w.pkt_payload = pkt_payload;
    if (w.ppp.b == 0) return -1;
    memset(pkt_exps, 0, w.ppp.B + w.ppp.b);
    memset(pkt_payload, 0, (w.ppp.B + w.ppp.b) * P * 4);
    worker_run(&w);
    return w.rc;
}

/* glibc srandom_r/random_r, TYPE_3 (degree 31, separation 3) — the generator
 * behind rand() that the reference's benchmarks seed with srand(seed). */
void orc_glibc_rand(uint32_t seed, uint64_t n, int32_t* out) {
    int32_t r[34];
    int64_t word;
    if (seed == 0) seed = 1;
    r[0] = (int32_t)seed;
    for (int i = 1; i < 31; i++) {
        int64_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
        word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r[i] = (int32_t)word;
    }
    /* ring of the last 34 values; discard the first 310 outputs */
    uint32_t ring[34];
    for (int i = 0; i < 31; i++) ring[i] = (uint32_t)r[i];
    for (int i = 31; i < 34; i++) ring[i] = ring[i - 31];
    uint64_t k = 34;
    for (uint64_t i = 0; i < 310 + n; i++, k++) {
        uint32_t v = ring[(k - 31) % 34] + ring[(k - 3) % 34];
        ring[k % 34] = v;
        if (i >= 310) out[i - 310] = (int32_t)(v >> 1);
    }
}

void orc_ref_random_floats(uint32_t seed, uint64_t n, float* out) {
    int32_t* r = (int32_t*)malloc(n * sizeof(int32_t));
    if (!r) return;
    orc_glibc_rand(seed, n, r);
    for (uint64_t i = 0; i < n; i++) {
        int32_t v = r[i];
        uint32_t bits = ((uint32_t)(v % 2) << 31) | ((uint32_t)(v % 254) << 23) | (uint32_t)(v % (1 << 23));
        memcpy(&out[i], &bits, 4);
    }
    free(r);
}

/* ------------------------------------------------------------------------ */
/* DPDK frames.                                               */

uint16_t orc_pkt_id_to_pool_index(uint64_t pkt_id, uint32_t start, uint32_t shift, uint32_t mop) {
    /* dpdk_worker_thread_utils.inc:42-52 */
    uint32_t i = (uint32_t)((pkt_id + shift) % (2ull * mop));
    if (i < mop) return (uint16_t)(start + i);
    return (uint16_t)((start + (i - mop)) | 0x8000);
}

/* rte_raw_cksum over a buffer: sum of the 16-bit words as they sit in memory
 * (little-endian host), folded twice; rte_ipv4_phdr_cksum returns it as is. */
static uint16_t raw_cksum(const uint8_t* b, size_t len) {
    uint32_t sum = 0;
    for (size_t i = 0; i + 1 < len; i += 2) sum += (uint32_t)b[i] | ((uint32_t)b[i + 1] << 8);
    if (len & 1) sum += b[len - 1];
    sum = (sum & 0xffff) + (sum >> 16);
    sum = (sum & 0xffff) + (sum >> 16);
    return (uint16_t)sum;
}

static void put16be(uint8_t* p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

/* Frame p's headers (BuildPacket, dpdk_worker_thread_utils.inc:73-126):
 * Ethernet, IPv4, UDP (pseudo-header checksum), SwitchML header; returns the
 * SwitchML header (extra info at +8, entries at +10).  The frame is zeroed
 * first: bytes the reference leaves stale are written as 0. */
static uint8_t* frame_header(uint8_t* f, uint64_t p, uint64_t P, uint64_t data_len, const orc_frame_params* prm) {
    memset(f, 0, data_len);
    /* 1. Ethernet */
    memcpy(f + 0, prm->dst_mac, 6);
    memcpy(f + 6, prm->src_mac, 6);
    put16be(f + 12, 0x0800);
    /* 2. IPv4 */
    uint8_t* ip = f + 14;
    ip[0] = 0x45;
    put16be(ip + 2, (uint16_t)(data_len - 14));
    ip[8] = 128;          /* ttl */
    ip[9] = 17;           /* IPPROTO_UDP */
    memcpy(ip + 12, &prm->src_ip_be, 4);
    memcpy(ip + 16, &prm->dst_ip_be, 4);
    /* 3. UDP */
    uint8_t* udp = ip + 20;
    memcpy(udp + 0, &prm->src_port_be, 2);
    memcpy(udp + 2, &prm->dst_port_be, 2);
    put16be(udp + 4, (uint16_t)(data_len - 34));
    uint8_t psd[12];
    memcpy(psd + 0, ip + 12, 4);
    memcpy(psd + 4, ip + 16, 4);
    psd[8] = 0;
    psd[9] = ip[9];
    put16be(psd + 10, (uint16_t)(data_len - 14 - 20)); /* l3 len - ihl*4 */
    uint16_t ck = raw_cksum(psd, 12);
    memcpy(udp + 6, &ck, 2);
    /* 4. SwitchML header */
    uint8_t* h = udp + 8;
    uint8_t len_enum = P < 64 ? 0 : P < 128 ? 1 : P < 256 ? 2 : 3;
    h[0] = (uint8_t)((1 << 4) + len_enum);
    h[1] = (uint8_t)prm->job_id;
    uint32_t pid = (uint32_t)p;
    memcpy(h + 2, &pid, 4); /* host order */
    put16be(h + 6, orc_pkt_id_to_pool_index(p, prm->pool_index_start, prm->pool_index_shift,
                                            prm->max_outstanding_pkts));
    return h;
}

/* INT32 jobs (DataType::INT32): no extra batch (NeedsExtraBatch is false for
 * INT32, ppp.cc:65-67), so B frames; frame p = BuildPacket's headers + the
 * INT32 PreprocessSingle of block p (ppp.cc:158-190: htonl of each word, only
 * the n real words; the extra-info bytes are left as they were — 0 here). */
int orc_build_frames_i32(const int32_t* in, uint64_t numel, uint64_t P, const orc_frame_params* prm,
                         uint8_t* frames, uint64_t stride) {
    const uint64_t B = orc_num_blocks(numel, P);
    const uint64_t data_len = 14 + 20 + 8 + 8 + P * 4 + 2;
    if (stride < data_len) return -1;
    for (uint64_t p = 0; p < B; p++) {
        uint8_t* entries = frame_header(frames + p * stride, p, P, data_len, prm) + 10;
        const uint64_t off = p * P, n = numel - off < P ? numel - off : P;
        for (uint64_t i = 0; i < n; i++) {
            uint32_t w = bswap32((uint32_t)in[off + i]);
            memcpy(entries + 4 * i, &w, 4);
        }
    }
    return 0;
}

/* The receive loop for an INT32 job slice (dpdk_worker_thread.cc:300-345):
 * discard a pkt_id already received or a frame of another job, otherwise
 * PostprocessSingle's INT32 branch (ppp.cc:262-298): ntohl of the n real
 * words of block pkt_id into out.  pkt_id >= B is counted as discarded.
 * `seen` (one byte per pkt_id, B) carries over between calls of one slice. */
void orc_unpack_frames_i32(const uint8_t* frames, uint64_t num_frames, uint64_t stride, uint64_t numel,
                           uint64_t P, uint64_t job_id, uint8_t* seen, int32_t* out, uint64_t counts[2]) {
    const uint64_t B = orc_num_blocks(numel, P);
    for (uint64_t f = 0; f < num_frames; f++) {
        const uint8_t* fr = frames + f * stride;
        uint32_t pid;
        memcpy(&pid, fr + 44, 4);
        if (pid >= B || seen[pid] || fr[43] != (uint8_t)job_id) {
            counts[1]++;
            continue;
        }
        seen[pid] = 1;
        counts[0]++;
        const uint64_t off = (uint64_t)pid * P, n = numel - off < P ? numel - off : P;
        for (uint64_t i = 0; i < n; i++) {
            uint32_t w;
            memcpy(&w, fr + 52 + 4 * i, 4);
            out[off + i] = (int32_t)bswap32(w);
        }
    }
}

int orc_build_frames(const float* in, uint64_t numel, uint64_t P, uint16_t W, const int8_t* global_exps,
                     uint32_t batch_max, const orc_frame_params* prm, uint8_t* frames, uint64_t stride) {
    const uint64_t B = orc_num_blocks(numel, P);
    const uint64_t b = B < batch_max ? B : batch_max;
    const uint64_t data_len = 14 + 20 + 8 + 8 + P * 4 + 2;
    if (stride < data_len) return -1;
    float lut[256];
    orc_scale_lut(W, lut);
    for (uint64_t p = 0; p < B + b; p++) {
        uint8_t* h = frame_header(frames + p * stride, p, P, data_len, prm);
        /* PreprocessSingle(p, entries = h + 10, extra = h + 8) — ppp.cc:69-156 */
        uint8_t* extra = h + 8;
        uint8_t* entries = h + 10;
        if (p >= b) {
            uint64_t k = p - b, off = k * P, n = numel - off < P ? numel - off : P;
            int8_t e = global_exps ? global_exps[k] : orc_block_exponent(in + off, n);
            float sc = lut[(uint8_t)e];
            for (uint64_t i = 0; i < n; i++) {
                uint32_t w = orc_quantize_value(in[off + i], sc);
                memcpy(entries + 4 * i, &w, 4);
            }
        }
        if (p < B) {
            uint64_t off = p * P, n = numel - off < P ? numel - off : P;
            extra[0] = (uint8_t)orc_block_exponent(in + off, n);
        }
    }
    return 0;
}

/* Receive loop of DpdkWorkerThread (dpdk_worker_thread.cc:300-345), one frame
 * at a time in the given order: discard a pkt_id already received (the rx
 * bitmap, :316-322) or a frame of another job (short_job_id, :325-331);
 * otherwise PostprocessSingle(pkt_id, frame + 52, frame + 50) (ppp.cc:197-260):
 * dequantize block pkt_id - b with scaling_factors_[pkt_id - b] when pkt_id >= b,
 * then, if pkt_id < B, scaling_factors_[pkt_id] from the exponent byte.
 * pkt_id >= B + b is counted as discarded (the reference would index its
 * bitmap out of range).  `exps` (int8[B]) and `seen` (the rx bitmap, one
 * byte per pkt_id, B + b, zeroed by the caller per slice) carry over between
 * calls; the scale is recomputed from exps (scaling_factors_[k] is exactly
 * orc_scale(W, exps[k])). */
void orc_dequantize_frames(const uint8_t* frames, uint64_t num_frames, uint64_t stride, uint64_t numel,
                           uint64_t P, uint16_t W, uint32_t batch_max, uint64_t job_id, int8_t* exps,
                           uint8_t* seen, float* out, uint64_t counts[2]) {
    const uint64_t B = orc_num_blocks(numel, P);
    const uint64_t b = B < batch_max ? B : batch_max;
    const uint64_t total = B + b;
    float lut[256];
    orc_scale_lut(W, lut);
    for (uint64_t f = 0; f < num_frames; f++) {
        const uint8_t* fr = frames + f * stride;
        uint32_t pid;
        memcpy(&pid, fr + 44, 4);
        if (pid >= total || seen[pid] || fr[43] != (uint8_t)job_id) {
            counts[1]++;
            continue;
        }
        seen[pid] = 1;
        counts[0]++;
        if (pid >= b) {
            const uint64_t k = pid - b, off = k * P, n = numel - off < P ? numel - off : P;
            const float s = lut[(uint8_t)exps[k]];
            for (uint64_t i = 0; i < n; i++) {
                uint32_t w;
                memcpy(&w, fr + 52 + 4 * i, 4);
                out[off + i] = orc_dequantize_value(w, s);
            }
        }
        if (pid < B) exps[pid] = (int8_t)fr[50];
    }
}

