// Host cost of the calls the client makes per job: hipPointerGetAttributes
// (device / pinned / pageable pointers), hipEventRecord, hipEventQuery, and
// an empty-ish kernel launch through sml_roundtrip_loopback_batch (1 slice).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "switchml_hip.h"

template <class F>
static double per_call_us(F f, int n = 20000) {
    for (int i = 0; i < 100; i++) f();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) f();
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
}

int main() {
    void *d, *h;
    (void)hipMalloc(&d, 1 << 20);
    (void)hipHostMalloc(&h, 1 << 20, hipHostMallocDefault);
    std::vector<char> pg(1 << 20);
    hipPointerAttribute_t a;
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    hipStream_t st;
    (void)hipStreamCreate(&st);
    printf("{\"hipPointerGetAttributes_device_us\": %.3f,", per_call_us([&] { (void)hipPointerGetAttributes(&a, d); }));
    printf(" \"hipPointerGetAttributes_pinned_us\": %.3f,", per_call_us([&] { (void)hipPointerGetAttributes(&a, h); }));
    printf(" \"hipPointerGetAttributes_pageable_us\": %.3f,", per_call_us([&] {
               if (hipPointerGetAttributes(&a, pg.data()) != hipSuccess) (void)hipGetLastError();
           }));
    printf(" \"hipEventRecord_us\": %.3f,", per_call_us([&] { (void)hipEventRecord(ev, st); }));
    (void)hipStreamSynchronize(st);
    printf(" \"hipEventQuery_done_us\": %.3f,", per_call_us([&] { (void)hipEventQuery(ev); }));
    sml_slice s{static_cast<const float*>(d), static_cast<float*>(d), 1024};
    printf(" \"batch_launch_1slice_us\": %.3f,", per_call_us([&] { (void)sml_roundtrip_loopback_batch(&s, 1, 256, 2, 0, st); }, 2000));
    (void)hipStreamSynchronize(st);
    sml_slice s4[4];
    for (int i = 0; i < 4; i++) s4[i] = sml_slice{static_cast<const float*>(d) + 1024 * i, static_cast<float*>(d) + 1024 * i, 1024};
    printf(" \"batch_launch_4slices_us\": %.3f}\n", per_call_us([&] { (void)sml_roundtrip_loopback_batch(s4, 4, 256, 2, 0, st); }, 2000));
    (void)hipStreamSynchronize(st);
    return 0;
}
