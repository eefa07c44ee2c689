/* capi_roundtrip.c — a plain C caller of the kernel C-ABI (include/switchml_hip.h),
 * the way a backend written in C (or bound through cgo/JNI) drives it: no C++,
 * no torch.  One job slice goes through the dummy backend's path in bulk:
 *   sml_quantize_pack (PreprocessSingle for every packet, ppp.cc:69-156)
 *   -> sml_loopback_aggregate (DummyBackend::ProcessPacket x W, dummy_backend.cc:72-84)
 *   -> sml_dequantize (PostprocessSingle, ppp.cc:194-260)
 * and the result is checked with the reference's own verify rule
 * (allreduce_benchmark/main.cc:343-356: out = in * W within 1 %, signed) and
 * the quantizer's error bound: out = W*q/s with s = 2^31 / (W * 2^e) and
 * |q - in*s| <= 1/2, so |out - W*in| <= W^2 * 2^(e-32), plus the float
 * rounding of the final division.
 * Usage: capi_roundtrip [numel] [packet_numel] [num_workers]  -> prints "capi ok"
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "switchml_hip.h"

#define HIPCK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
#define SMLCK(x) do { sml_status_t s_ = (x); if (s_ != SML_OK) { \
    fprintf(stderr, "%s failed: %s %s\n", #x, sml_status_string(s_), sml_last_error()); return 1; } } while (0)

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1000003;
    const uint32_t P = argc > 2 ? (uint32_t)atoi(argv[2]) : 256;
    const uint16_t W = argc > 3 ? (uint16_t)atoi(argv[3]) : 4;
    const uint64_t B = sml_num_blocks(n, P);
    float* x = (float*)malloc(n * sizeof(float));
    float* y = (float*)malloc(n * sizeof(float));
    int8_t* e = (int8_t*)malloc(B);
    if (!x || !y || !e) return 1;
    /* allreduce_benchmark's float pattern (main.cc:207-212), scaled to gradients */
    for (uint64_t i = 0; i < n; i++) x[i] = (float)(i % 1000) * ((i & 1) ? -1.0f : 1.0f) * 1e-3f;

    float *dx, *dy;
    int32_t* dpay;
    int8_t* dexp;
    hipStream_t st;
    HIPCK(hipStreamCreate(&st));
    HIPCK(hipMalloc((void**)&dx, n * sizeof(float)));
    HIPCK(hipMalloc((void**)&dy, n * sizeof(float)));
    HIPCK(hipMalloc((void**)&dpay, B * P * sizeof(int32_t)));
    HIPCK(hipMalloc((void**)&dexp, B));
    HIPCK(hipMemcpyAsync(dx, x, n * sizeof(float), hipMemcpyHostToDevice, st));

    SMLCK(sml_quantize_pack(dx, n, P, W, NULL, dpay, dexp, 0, st));
    SMLCK(sml_loopback_aggregate(dpay, B * P, W, 0, st));
    SMLCK(sml_dequantize(dpay, dexp, n, P, W, dy, 0, st));
    HIPCK(hipMemcpyAsync(y, dy, n * sizeof(float), hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(e, dexp, B, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));

    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; i++) {
        const float expected = x[i] * (float)W;
        const double bound = (double)W * W * ldexp(1.0, e[i / P] - 32) + fabs((double)expected) * 1.2e-7;
        const float err_pct = expected != 0.0f ? (expected - y[i]) / expected * 100.0f : 0.0f;
        if (err_pct > 1.0f || fabs((double)y[i] - (double)expected) > bound) bad++;
    }
    printf("capi %s: numel %llu packet_numel %u num_workers %u blocks %llu mismatches %llu\n",
           bad ? "FAILED" : "ok", (unsigned long long)n, P, W, (unsigned long long)B, (unsigned long long)bad);
    hipFree(dx); hipFree(dy); hipFree(dpay); hipFree(dexp); hipStreamDestroy(st);
    free(x); free(y); free(e);
    return bad ? 2 : 0;
}
